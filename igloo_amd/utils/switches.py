"""The environment switches the engine reads -- all of them, documented here.

Tuning values and code-path choices are module constants (tests set them
directly); what remains in the environment is deployment configuration,
the JIT / graph modes, and ONE debug namespace, ``IGLOO_DEBUG``: a comma
list of tokens (``token`` or ``token=value``), read by Python and C++ alike
(csrc/runtime/runtime.cpp ``debug_flag``):

==============================  =====================================================
``IGLOO_DEBUG`` token           effect
==============================  =====================================================
``key_tags``                    verify every readback-free key fact (uniqueness tags,
                                bounds) against the data (the GPU test suite sets it)
``sync_check``                  fail on an unexpected device synchronisation
``spec``                        print why a replayed readback recording diverged
``jit``                         generated-kernel (hiprtc) diagnostics
``jit_dump=<dir>``              write every generated kernel's source to <dir>
``fused``                       fused scan planner diagnostics
``graph_dump=<dir>``            DOT dump of every captured query graph
``collectives``                 record the engine call site of every collective
``roctx``                       roctx ranges per query / operator (rocprofv3 --marker-trace)
``sanitize``                    build the extension with host ASan / UBSan
``ff_mfma``                     interpreted fused aggregation on the MFMA one-hot kernel
                                (measured slower: profiles/r5_mfma_ab_counters.txt)
``ff_jit_mfma``                 the same inside generated scan kernels
``having_general``              sorted GROUP BY + HAVING on the run-folding kernel
                                instead of the streaming scan (agg.hip)
``like_nodword``                LIKE without the aligned-dword prefilter (strings.hip)
``no_templates``                plan every new statement text from scratch (no statement
                                templates, sql/template.py)
``no_agg_part``                 high-cardinality GROUP BY through global atomics instead
                                of the radix-partitioned LDS aggregate (ops/agg.py)
``agg_part_min128``             the partitioned aggregate only from 128 buckets (fewer
                                buckets: global atomics instead of sliced buckets)
``no_mask_counts``              generated scan masks without per-tile counts (the
                                selection counts the mask again, ops/select.py)
``pack_bits_scalar``            composite-key packing one row per lane instead of four
                                with 16-byte loads (util.hip pack_bits)
==============================  =====================================================

Other variables (each read in one place):

* ``IGLOO_LOG``: log level; ``IGLOO_FAULT``: fault injection (utils/faults.py);
* ``IGLOO_JIT`` (``async`` | ``sync`` | ``off``), ``IGLOO_JIT_CACHE``, ``IGLOO_JIT_AOT``:
  generated kernels (ops/jit.py); ``IGLOO_OFFLOAD_ARCH``: build target (gfx950);
* ``IGLOO_GRAPHS``: query graphs on / off (exec/graphs.py);
* ``IGLOO_FORCE_SPMD``, ``IGLOO_COMM_BACKEND``: SPMD rehearsal on one GPU, backend;
* ``IGLOO_DEVICE_BUDGET_GB``, ``IGLOO_HBM_BUDGET_GB``, ``IGLOO_PACK_BUDGET_GB``:
  device memory budgets;
* ``IGLOO_PARQUET_READ_THREADS``, ``IGLOO_PARQUET_BATCH_BYTES``: cold-scan I/O;
* ``IGLOO_SUPERVISOR_ID``: set by the node supervisor for its workers;
* ``IGLOO_<setting>`` for every field of utils/config.py ``IglooConfig``.
"""
from __future__ import annotations

import os
from typing import Dict, Optional


def _parse(raw: Optional[str]) -> Dict[str, str]:
    out: Dict[str, str] = {}
    for tok in (raw or "").split(","):
        tok = tok.strip()
        if not tok:
            continue
        k, _, v = tok.partition("=")
        out[k.strip().lower()] = v.strip() or "1"
    return out


DEBUG: Dict[str, str] = _parse(os.environ.get("IGLOO_DEBUG"))

ENV = ("IGLOO_DEBUG", "IGLOO_LOG", "IGLOO_FAULT", "IGLOO_JIT", "IGLOO_JIT_CACHE", "IGLOO_JIT_AOT",
       "IGLOO_OFFLOAD_ARCH", "IGLOO_GRAPHS", "IGLOO_FORCE_SPMD", "IGLOO_COMM_BACKEND", "IGLOO_DEVICE_BUDGET_GB",
       "IGLOO_HBM_BUDGET_GB", "IGLOO_PACK_BUDGET_GB", "IGLOO_PARQUET_READ_THREADS", "IGLOO_PARQUET_BATCH_BYTES",
       "IGLOO_SUPERVISOR_ID")


def debug(token: str) -> bool:
    return token in DEBUG


def debug_value(token: str) -> Optional[str]:
    return DEBUG.get(token)
