"""Runtime for query-specialised kernels (csrc/runtime/jit.cpp).

A code generator (e.g. ``exec/fused_jit.py``) emits HIP source for one plan
shape; this module compiles it for gfx950 with hiprtc, keeps the code object
(in memory and on disk, keyed by a hash of the source), loads it into the HIP
context and launches it with a flat 8-byte-slot kernarg buffer.

Compilation is adaptive (``IGLOO_JIT``):

* ``async`` (default): the first request of a source submits the compile to a
  background thread and returns ``None`` - the caller runs its interpreted
  kernel; once the code object is ready, later executions of the same plan
  shape use the generated kernel (like a prepared statement's cached plan).
  A code object already on disk is loaded at once.
* ``sync``: compile on first use and wait (tests; deterministic paths).
* ``off``: never generate code.

hiprtc runs on the host without a device, so compilation overlaps GPU work.
The reference has no code generation: DataFusion interprets its physical
plan through Arrow compute kernels (reference crates/engine/src/lib.rs:55-56).
"""
from __future__ import annotations

from ..utils import switches as _sw
import concurrent.futures as cf
import hashlib
import os
import threading
from pathlib import Path
from typing import Dict, List, Optional, Sequence

from ._lib import KERNEL_CALLS, check_not_capturing, native

MODE = os.environ.get("IGLOO_JIT", "async").lower()
ARCH = "gfx950"
_VERSION = "1"  # bump when the compile options or the kernarg convention change
CACHE_DIR = Path(os.environ.get("IGLOO_JIT_CACHE", os.path.join(os.environ.get("TMPDIR", "/tmp"), "igloo_jit")))
#: ahead-of-time code objects shipped with the build (read-only, searched
#: first): the query-specialised kernels of the TPC-H suite at the benchmark
#: scale, compiled by ``scripts/gpu_run.sh jitcache`` so a fresh process does
#: not pay for hiprtc in its first (cold) queries. A source not found here or
#: in CACHE_DIR compiles on demand as usual.
AOT_DIR = Path(os.environ.get("IGLOO_JIT_AOT", os.path.join(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))), "_jit_cache")))
#: generated-kernel SOURCES recorded from the benchmark suite (committed text):
#: ``build()`` (igloo_amd/_build.py ``build_aot``) compiles each into AOT_DIR
#: with hiprtc on the build host -- no GPU needed -- so the code objects are
#: our own build output, not checked-in binaries
AOT_SOURCES = Path(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "jit_sources"))
#: IGLOO_DEBUG=jit_dump=<dir>: write every generated kernel's source there (how
#: AOT_SOURCES is recorded: scripts/gpu_run.sh jitsources)
DUMP_DIR = _sw.debug_value("jit_dump")

_lock = threading.Lock()
_kernels: Dict[str, "JitKernel"] = {}
_pending: Dict[str, cf.Future] = {}
_failed: Dict[str, str] = {}
_names: Dict[str, str] = {}
_pool: Optional[cf.ThreadPoolExecutor] = None
STATS = {"compiled": 0, "disk_hits": 0, "launches": 0, "fallbacks": 0, "failed": 0}


class JitKernel:
    __slots__ = ("name", "handle", "key")

    def __init__(self, name: str, handle: int, key: str):
        self.name, self.handle, self.key = name, handle, key

    def launch(self, grid: int, block: int, shmem: int, stream: int, args: Sequence[int]) -> None:
        STATS["launches"] += 1
        KERNEL_CALLS["jit:" + self.name] += 1
        native().jit_launch(self.handle, int(grid), int(block), int(shmem), int(stream),
                            [int(a) & 0xFFFFFFFFFFFFFFFF for a in args])

    def attributes(self) -> dict:
        return native().jit_attributes(self.handle)


def enabled() -> bool:
    return MODE in ("async", "sync")


def _key(src: str, name: str) -> str:
    return hashlib.sha256(f"{_VERSION}|{ARCH}|{name}|{src}".encode()).hexdigest()[:32]


def _disk_path(key: str) -> Path:
    return CACHE_DIR / f"{key}.co"


def _compile(src: str, name: str, key: str) -> bytes:
    code = native().jit_compile(src, name, ARCH)
    try:
        CACHE_DIR.mkdir(parents=True, exist_ok=True)
        tmp = _disk_path(key).with_suffix(f".{os.getpid()}.tmp")
        tmp.write_bytes(code)
        os.replace(tmp, _disk_path(key))
    except OSError:
        pass
    STATS["compiled"] += 1
    return code


def _load(code: bytes, name: str, key: str) -> JitKernel:
    check_not_capturing("generated-kernel load")   # module loads are not graph operations
    k = JitKernel(name, native().jit_load(code, name), key)
    _kernels[key] = k
    return k


def get(src: str, name: str, mode: Optional[str] = None) -> Optional[JitKernel]:
    """The compiled kernel for ``src`` (entry point ``name``), or None while
    it is being compiled / when generation is off or failed."""
    mode = mode or MODE
    if mode not in ("async", "sync"):
        return None
    key = _key(src, name)
    k = _kernels.get(key)
    if k is not None:
        return k
    if DUMP_DIR:
        _dump(src, name, key)
    with _lock:
        k = _kernels.get(key)
        if k is not None:
            return k
        if key in _failed:
            STATS["fallbacks"] += 1
            return None
        fut = _pending.get(key)
        if fut is None:
            p = AOT_DIR / f"{key}.co"
            if not p.exists():
                p = _disk_path(key)
            if p.exists():
                try:
                    STATS["disk_hits"] += 1
                    return _load(p.read_bytes(), name, key)
                except Exception:   # stale / truncated cache entry: recompile
                    if p.parent != AOT_DIR:
                        p.unlink(missing_ok=True)
            if mode == "sync":
                try:
                    return _load(_compile(src, name, key), name, key)
                except Exception as e:
                    _failed[key] = str(e)
                    STATS["failed"] += 1
                    raise
            global _pool
            if _pool is None:
                _pool = cf.ThreadPoolExecutor(max_workers=2,
                                              thread_name_prefix="igloo-jit")
            _pending[key] = _pool.submit(_compile, src, name, key)
            _names[key] = name
            STATS["fallbacks"] += 1
            return None
        if not fut.done():
            STATS["fallbacks"] += 1
            return None
        del _pending[key]
        try:
            code = fut.result()
        except Exception as e:   # a generator bug must not take the query down: keep interpreting
            _failed[key] = str(e)
            STATS["failed"] += 1
            if _sw.debug("jit"):
                print(f"[jit] {name}: compile failed:\n{e}\n{src}", flush=True)
            return None
        return _load(code, name, key)


def _dump(src: str, name: str, key: str) -> None:
    try:
        d = Path(DUMP_DIR)
        d.mkdir(parents=True, exist_ok=True)
        p = d / f"{key}.hip"
        if not p.exists():
            p.write_text(f"// igloo-jit-kernel: {name}\n{src}")
    except OSError:
        pass


def aot_compile(sources: Path = AOT_SOURCES, out: Path = AOT_DIR, jobs: int = 8) -> dict:
    """Compile every recorded generated-kernel source (``<key>.hip`` with a
    ``// igloo-jit-kernel: <entry>`` first line) into ``out/<key>.co`` with
    hiprtc for gfx950. Incremental: a code object newer than its source is
    kept. Returns counts."""
    stats = {"sources": 0, "compiled": 0, "kept": 0, "failed": 0}
    if not sources.is_dir():
        return stats
    out.mkdir(parents=True, exist_ok=True)
    todo = []
    for p in sorted(sources.glob("*.hip")):
        stats["sources"] += 1
        text = p.read_text()
        first, _, src = text.partition("\n")
        if not first.startswith("// igloo-jit-kernel: "):
            stats["failed"] += 1
            continue
        name = first.split(": ", 1)[1].strip()
        key = _key(src, name)
        co = out / f"{key}.co"
        if co.exists() and co.stat().st_mtime >= p.stat().st_mtime:
            stats["kept"] += 1
            continue
        todo.append((src, name, co))

    def one(job):
        src, name, co = job
        code = native().jit_compile(src, name, ARCH)
        tmp = co.with_suffix(f".{os.getpid()}.tmp")
        tmp.write_bytes(code)
        os.replace(tmp, co)
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for f in [ex.submit(one, j) for j in todo]:
            try:
                f.result()
                stats["compiled"] += 1
            except Exception:   # noqa: BLE001 - that shape compiles on demand at run time
                stats["failed"] += 1
    return stats


def wait_all(timeout: Optional[float] = None) -> None:
    """Block until every submitted compile finished, then load them all (so
    the set of generated kernels changes at one point, not query by query)."""
    with _lock:
        futs = list(_pending.values())
    cf.wait(futs, timeout=timeout)
    with _lock:
        for key, fut in list(_pending.items()):
            if not fut.done():
                continue
            del _pending[key]
            try:
                code = fut.result()
            except Exception as e:   # noqa: BLE001 - recorded, the interpreted kernels stay
                _failed[key] = str(e)
                STATS["failed"] += 1
                continue
            name = _names.get(key, "")
            if name:
                _load(code, name, key)


def failures() -> List[str]:
    return list(_failed.values())


def generation() -> Optional[int]:
    """Identifies the set of generated kernels a query can use: the number
    loaded plus the number failed, or None while compiles are in flight (the
    set is about to change). A query graph (exec/graphs.py) captured under
    one generation is re-captured under the next."""
    with _lock:
        if _pending:
            return None
        return len(_kernels) + len(_failed)
