"""Communicator: one process per GPU, collectives over RCCL (xGMI) via
``torch.distributed`` ("nccl" backend == RCCL on ROCm), gloo on CPU.

The reference has no collective layer at all — every inter-process call is a
gRPC/Flight RPC and the shuffle is declared but never implemented (reference
crates/api/proto/coordinator.proto:50-58 "for shuffle", worker returns empty
bytes at crates/worker/src/service.rs:26-32). SURVEY §2.5 M5/§5.8.

xGMI is a full mesh of point-to-point links, so data exchanges use
all-to-all-v (every peer sends directly on its own link) and all-gather-v,
never ring-style reductions of large buffers; small control values (counts,
sizes, NDVs) are batched into one tiny all-reduce / all-gather.
"""
from __future__ import annotations

from ..utils import switches as _sw
import datetime
import os
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from ..ops._lib import device_ints, to_host_f64s, to_host_ints
from ..utils import faults
from ..utils.errors import CommError
from ..utils.log import get_logger

log = get_logger("comm")


class Communicator:
    def __init__(self, rank: int, world_size: int, device, group=None, backend: str = "nccl",
                 force_spmd: bool = False):
        self.rank = rank
        self.world_size = world_size
        #: rows are spread over ranks and exchanges run. ``force_spmd`` keeps it
        #: on for a world of one: every exchange and collective then really runs
        #: (RCCL / gloo with one rank) — the single-GPU rehearsal of the
        #: multi-GPU code path, including collectives inside query graphs
        self.spmd = world_size > 1 or force_spmd
        self.device = torch.device(device)
        self.group = group
        self.backend = backend
        # gloo moves host tensors only: device data is staged through the host
        # (used to rehearse multi-rank GPU code paths on a single GPU)
        self.wire = torch.device("cpu") if backend == "gloo" else self.device
        self.bytes_sent = 0
        self.calls = 0
        self.chunk_calls = 0     # of ``calls``: the 2nd.. chunks of pipelined exchanges (one logical exchange each)
        self.trace = [] if _sw.debug("collectives") else None

    # ------------------------------------------------------------- lifecycle
    @staticmethod
    def init(backend: Optional[str] = None, device=None, timeout_s: float = 600.0,
             force_spmd: Optional[bool] = None) -> "Communicator":
        """Initialise from torchrun-style env (RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT).
        ``force_spmd`` (default: env IGLOO_FORCE_SPMD=1) runs the SPMD path
        even for a world of one."""
        rank = int(os.environ.get("RANK", "0"))
        world = int(os.environ.get("WORLD_SIZE", "1"))
        local = int(os.environ.get("LOCAL_RANK", str(rank)))
        if device is None:
            device = f"cuda:{local}" if torch.cuda.is_available() else "cpu"
        device = torch.device(device)
        if backend is None:
            backend = os.environ.get("IGLOO_COMM_BACKEND") or ("nccl" if device.type == "cuda" else "gloo")
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if not dist.is_initialized():
            kw = {}
            if device.type == "cuda":
                torch.cuda.set_device(device)
                if backend == "nccl":
                    kw["device_id"] = device
            dist.init_process_group(backend, rank=rank, world_size=world,
                                    timeout=datetime.timedelta(seconds=timeout_s), **kw)
        if force_spmd is None:
            force_spmd = os.environ.get("IGLOO_FORCE_SPMD") == "1"
        return Communicator(dist.get_rank(), dist.get_world_size(), device, None, backend, force_spmd)

    def abort(self):
        """Tear the data communicator down without a collective (a peer died):
        RCCL ops blocked on the dead rank return an error instead of waiting
        for the collective timeout."""
        if not dist.is_initialized():
            return
        try:
            from torch.distributed import distributed_c10d as c10d
            if hasattr(c10d, "_abort_process_group"):
                c10d._abort_process_group(self.group or c10d.GroupMember.WORLD)
        except Exception as e:  # noqa: BLE001 - gloo groups have no abort: TCP resets end their ops
            log.warning("communicator abort: %s", e)

    def shutdown(self):
        """Barrier, then destroy the process group. Query graphs that captured
        RCCL collectives must be released first (QueryEngine.close): while one
        lives, destroy_process_group does not return."""
        if dist.is_initialized():
            try:
                self._count()
                dist.barrier()
            except Exception:  # pragma: no cover
                pass
            if self.device.type == "cuda":
                import gc
                gc.collect()
                torch.cuda.synchronize(self.device)
            dist.destroy_process_group()

    # ------------------------------------------------------------ primitives
    def _t(self, x, dtype=torch.int64) -> torch.Tensor:
        if self.wire.type == "cuda":
            return device_ints(x, self.wire, dtype)     # no sync; capture-safe
        return torch.as_tensor(x, dtype=dtype, device=self.wire)

    def _count(self):
        """One collective issued (``calls``); IGLOO_DEBUG=collectives also
        records the engine call site that issued it (``trace``)."""
        self.calls += 1
        if self.trace is not None:
            import traceback
            st = [f for f in traceback.extract_stack()[:-2] if "parallel/comm.py" not in f.filename]
            site = " <- ".join(f"{f.filename.split('igloo_amd/')[-1]}:{f.lineno}({f.name})" for f in st[-3:][::-1])
            self.trace.append(site)

    def barrier(self):
        if faults.ACTIVE:
            faults.check("comm_timeout", "barrier")
        if self.spmd:
            self._count()
            dist.barrier(group=self.group)

    def allreduce_int(self, x: int) -> int:
        if faults.ACTIVE:
            faults.check("comm_timeout", "allreduce_int")
        if not self.spmd:
            return int(x)
        t = self._t([int(x)])
        self._count()
        dist.all_reduce(t, group=self.group)
        return to_host_ints(t)[0]

    def allreduce_ints(self, xs: Sequence[int]) -> List[int]:
        if faults.ACTIVE:
            faults.check("comm_timeout", "allreduce_ints")
        if not self.spmd:
            return [int(x) for x in xs]
        t = self._t([int(x) for x in xs])
        self._count()
        dist.all_reduce(t, group=self.group)
        return to_host_ints(t)

    def allreduce_max_float(self, x: float) -> float:
        if faults.ACTIVE:
            faults.check("comm_timeout", "allreduce_max_float")
        if not self.spmd:
            return float(x)
        t = self._t([float(x)], torch.float64)
        self._count()
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return to_host_f64s(t)[0]

    def allreduce_max_tensor(self, t: torch.Tensor) -> torch.Tensor:
        """Element-wise max over ranks (in a 32-bit copy: portable across backends)."""
        if faults.ACTIVE:
            faults.check("comm_timeout", "allreduce_max_tensor")
        if not self.spmd:
            return t
        w = t.to(device=self.wire, dtype=torch.int32)
        self._count()
        dist.all_reduce(w, op=dist.ReduceOp.MAX, group=self.group)
        return w.to(device=t.device, dtype=t.dtype)

    def allreduce_tensor(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        """Element-wise SUM / MIN / MAX over ranks of an int64 / float64 tensor."""
        if faults.ACTIVE:
            faults.check("comm_timeout", "allreduce_tensor")
        if not self.spmd:
            return t
        w = t.contiguous().to(self.wire)
        if w is t:
            w = w.clone()
        self._count()
        dist.all_reduce(w, op={"sum": dist.ReduceOp.SUM, "min": dist.ReduceOp.MIN, "max": dist.ReduceOp.MAX}[op],
                        group=self.group)
        self.bytes_sent += w.numel() * w.element_size()
        return w.to(t.device)

    def reduce_scatter_tensor(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        """``t`` is [world, ...]: every rank contributes all of it and receives
        the element-wise SUM / MIN / MAX over ranks of block ``t[rank]`` only
        (partitioned aggregates: each rank keeps the states of the keys it
        owns; RCCL moves (world-1)/world of the bytes an all-reduce would
        hand every rank)."""
        if faults.ACTIVE:
            faults.check("comm_timeout", "reduce_scatter_tensor")
        assert t.shape[0] == self.world_size, (t.shape, self.world_size)
        if not self.spmd:
            return t[0]
        src = t.contiguous().to(self.wire).reshape(-1)        # [world * block], block-major
        out = torch.empty(src.numel() // self.world_size, dtype=src.dtype, device=self.wire)
        self._count()
        dist.reduce_scatter_tensor(out, src, op={"sum": dist.ReduceOp.SUM, "min": dist.ReduceOp.MIN,
                                                  "max": dist.ReduceOp.MAX}[op], group=self.group)
        self.bytes_sent += src.numel() * src.element_size() * (self.world_size - 1) // max(self.world_size, 1)
        return out.view(tuple(t.shape[1:])).to(t.device)

    def allgather_ints(self, xs: Sequence[int]) -> List[List[int]]:
        """Every rank contributes len(xs) ints; returns [rank][i]."""
        if faults.ACTIVE:
            faults.check("comm_timeout", "allgather_ints")
        k = len(xs)
        if not self.spmd:
            return [list(map(int, xs))]
        t = self._t([int(x) for x in xs])
        out = torch.empty(self.world_size * k, dtype=torch.int64, device=self.wire)
        self._count()
        dist.all_gather_into_tensor(out, t, group=self.group)
        v = to_host_ints(out)
        return [v[r * k:(r + 1) * k] for r in range(self.world_size)]

    def allgather_tensor(self, t: torch.Tensor) -> torch.Tensor:
        """Every rank's equally sized ``t`` concatenated (rank order), on the
        data device; one all-gather (staged through the host under gloo)."""
        if faults.ACTIVE:
            faults.check("comm_timeout", "allgather_tensor")
        if not self.spmd:
            return t
        src = t.contiguous().to(self.wire)
        out = torch.empty((self.world_size * src.shape[0],) + tuple(src.shape[1:]), dtype=src.dtype, device=self.wire)
        self._count()
        dist.all_gather_into_tensor(out, src, group=self.group)
        self.bytes_sent += src.numel() * src.element_size() * (self.world_size - 1)
        return out.to(t.device)

    def allgather_object(self, obj) -> list:
        if faults.ACTIVE:
            faults.check("comm_timeout", "allgather_object")
        if not self.spmd:
            return [obj]
        out = [None] * self.world_size
        self._count()
        dist.all_gather_object(out, obj, group=self.group)
        return out

    def all_to_all_v(self, t: torch.Tensor, send_counts: Sequence[int],
                     recv_counts: Optional[Sequence[int]] = None) -> Tuple[torch.Tensor, List[int]]:
        """Rows of ``t`` grouped by destination (send_counts[r] rows to rank r)."""
        if faults.ACTIVE:
            faults.check("comm_timeout", "all_to_all_v")
        W = self.world_size
        if not self.spmd:
            return t, [t.shape[0]]
        if recv_counts is None:
            m = self.all_to_all_counts(send_counts)
            recv_counts = m
        tail = tuple(t.shape[1:])
        out = torch.empty((sum(recv_counts),) + tail, dtype=t.dtype, device=self.wire)
        src = t.contiguous().to(self.wire)
        if src.dtype == torch.bool:
            src = src.view(torch.uint8)
            out = out.view(torch.uint8)
        self._count()
        dist.all_to_all_single(out, src, list(map(int, recv_counts)), list(map(int, send_counts)), group=self.group)
        self.bytes_sent += src.numel() * src.element_size()
        if t.dtype == torch.bool:
            out = out.view(torch.bool)
        return out.to(t.device), list(recv_counts)

    def all_to_all_v_async(self, t: torch.Tensor, send_counts: Sequence[int], recv_counts: Sequence[int]):
        """``all_to_all_v`` issued asynchronously (a pipelined exchange keeps
        packing the next chunk while this one moves): returns (output on the
        wire device, work handle); ``wait()`` the handle before reading."""
        if faults.ACTIVE:
            faults.check("comm_timeout", "all_to_all_v")
        tail = tuple(t.shape[1:])
        out = torch.empty((sum(recv_counts),) + tail, dtype=t.dtype, device=self.wire)
        src = t.contiguous().to(self.wire)
        self._count()
        work = dist.all_to_all_single(out, src, list(map(int, recv_counts)), list(map(int, send_counts)),
                                      group=self.group, async_op=True)
        self.bytes_sent += src.numel() * src.element_size()
        return out, work

    def all_to_all_counts(self, send_counts: Sequence[int]) -> List[int]:
        if faults.ACTIVE:
            faults.check("comm_timeout", "all_to_all_counts")
        W = self.world_size
        s = self._t(list(send_counts))
        r = torch.empty(W, dtype=torch.int64, device=self.wire)
        self._count()
        dist.all_to_all_single(r, s, group=self.group)
        return to_host_ints(r)

    def all_to_all_matrix(self, rows: Sequence[Sequence[int]]) -> List[List[int]]:
        """rows[r] = k ints for peer r; returns [r][k] received from every peer
        (row counts and string byte counts of a shuffle in ONE exchange)."""
        if faults.ACTIVE:
            faults.check("comm_timeout", "all_to_all_counts")
        W = self.world_size
        k = len(rows[0]) if rows else 0
        if not self.spmd:
            return [list(map(int, r)) for r in rows]
        s = self._t([int(x) for r in rows for x in r])
        r = torch.empty(W * k, dtype=torch.int64, device=self.wire)
        self._count()
        dist.all_to_all_single(r, s, group=self.group)
        v = to_host_ints(r)
        return [v[i * k:(i + 1) * k] for i in range(W)]

    def all_gather_v(self, t: torch.Tensor, counts: Optional[List[int]] = None) -> Tuple[torch.Tensor, List[int]]:
        """Concatenate every rank's ``t`` (variable row counts) on every rank.
        One all-gather of equal-sized blocks: each rank's rows padded to the
        largest count (no point-to-point ops, so the same single collective
        serves eager execution and RCCL query graphs), then the padding is
        dropped by one device gather when the counts differ."""
        if faults.ACTIVE:
            faults.check("comm_timeout", "all_gather_v")
        W = self.world_size
        if not self.spmd:
            return t, [t.shape[0]]
        if counts is None:
            counts = [c[0] for c in self.allgather_ints([t.shape[0]])]
        tail = tuple(t.shape[1:])
        src = t.contiguous().to(self.wire)
        if src.dtype == torch.bool:
            src = src.view(torch.uint8)
        mx = max(counts) if counts else 0
        total = sum(counts)
        if mx == 0:
            out = torch.empty((0,) + tail, dtype=src.dtype, device=self.wire)
        else:
            if src.shape[0] < mx:
                pad = torch.zeros((mx - src.shape[0],) + tail, dtype=src.dtype, device=self.wire)
                src = torch.cat([src, pad]) if src.shape[0] else pad
            blocks = torch.empty((W * mx,) + tail, dtype=src.dtype, device=self.wire)
            self._count()
            dist.all_gather_into_tensor(blocks, src, group=self.group)
            self.bytes_sent += src.numel() * src.element_size() * (W - 1)
            if all(c == mx for c in counts):
                out = blocks
            else:
                # rows [r * mx, r * mx + counts[r]) of every rank r
                starts = [r * mx for r in range(W)]
                dev = self.wire
                cnt = device_ints(counts, dev) if dev.type == "cuda" else torch.tensor(counts, dtype=torch.int64)
                st = device_ints(starts, dev) if dev.type == "cuda" else torch.tensor(starts, dtype=torch.int64)
                first = torch.cumsum(cnt, 0) - cnt
                idx = torch.repeat_interleave(st - first, cnt, output_size=total) + \
                    torch.arange(total, dtype=torch.int64, device=dev)
                out = blocks.index_select(0, idx)
        if t.dtype == torch.bool:
            out = out.view(torch.bool)
        return out.to(t.device), counts

    def _peer(self, r: int) -> int:
        """Global rank of group member ``r`` (P2P ops address global ranks)."""
        if self.group is None:
            return r
        return dist.get_global_rank(self.group, r)

    def broadcast_tensor(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if faults.ACTIVE:
            faults.check("comm_timeout", "broadcast_tensor")
        if self.spmd:
            w = t.to(self.wire)
            self._count()
            dist.broadcast(w, src, group=self.group)
            if w is not t:
                t.copy_(w)
        return t


class LocalComm(Communicator):
    """World of one (no process group): lets distributed code paths run unchanged."""

    def __init__(self, device="cpu"):
        super().__init__(0, 1, device, None, "local")
