"""Build the native extension ``igloo_amd/_native*.so`` with hipcc for gfx950.

The extension holds the C++ SQL frontend, the hand-written CDNA4 kernels and
the device runtime (csrc/). It is built in-tree (never pip-installed) so the
GPU box loads exactly this file. Compilation is incremental (content hash of
source + flags + headers) and parallel across translation units.

Usage: ``python -m igloo_amd._build [--force] [--jobs N]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
OBJ = ROOT / "build" / "obj"
ARCH = os.environ.get("IGLOO_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: the igloo native core needs ROCm's hipcc")


def ext_path() -> Path:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return ROOT / "igloo_amd" / f"_native{suffix}"


def _includes() -> list[str]:
    import pybind11

    return [f"-I{CSRC}", f"-I{sysconfig.get_paths()['include']}", f"-I{pybind11.get_include()}"]


def _sources() -> list[Path]:
    srcs = sorted(CSRC.rglob("*.cpp")) + sorted(CSRC.rglob("*.hip"))
    # csrc/tools/: standalone host programs (sanitizer driver), not extension units
    return [p for p in srcs if "tools" not in p.relative_to(CSRC).parts]


def _headers_digest() -> str:
    h = hashlib.sha256()
    for p in sorted(CSRC.rglob("*.h")):
        h.update(p.read_bytes())
    return h.hexdigest()


def _sanitize() -> str:
    """IGLOO_DEBUG=sanitize=address+undefined: host sanitizers for the build
    (the value's '+' separates sanitizers; bare ``sanitize`` = address,undefined)."""
    from .utils import switches
    v = switches._parse(os.environ.get("IGLOO_DEBUG")).get("sanitize")
    if not v:
        return ""
    return "address,undefined" if v == "1" else v.replace("+", ",")


def _flags(src: Path) -> list[str]:
    base = ["-O3", "-fPIC", "-std=c++17", "-Wall", "-Wno-unused-function", "-Wno-unused-variable",
            "-Wno-unused-result", "-fvisibility=hidden"]
    if _sanitize():
        # host-only sanitizers (GPU ASan is not available on the pool)
        base += [f"-Xarch_host", f"-fsanitize={_sanitize()}"]
    # hipcc treats .cpp as HIP too; give every unit the real target so no
    # default-arch device pass is compiled
    return base + ["-x", "hip", f"--offload-arch={ARCH}", "-munsafe-fp-atomics"]


def _compile(src: Path, hdr_digest: str, force: bool) -> Path:
    flags = _flags(src)
    key = hashlib.sha256(src.read_bytes() + " ".join(flags).encode() + hdr_digest.encode()).hexdigest()[:16]
    obj = OBJ / f"{src.stem}.{key}.o"
    if obj.exists() and not force:
        return obj
    for stale in OBJ.glob(f"{src.stem}.*.o"):
        stale.unlink()
    cmd = [hipcc(), *flags, *_includes(), "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, jobs: int | None = None, verbose: bool = False) -> Path:
    """Compile what changed and link; one process at a time (a file lock:
    parallel test workers and a manual build share build/obj)."""
    import fcntl
    OBJ.mkdir(parents=True, exist_ok=True)
    with open(OBJ / ".lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            return _build_locked(force, jobs, verbose)
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)


def _build_locked(force: bool, jobs: int | None, verbose: bool) -> Path:
    srcs = _sources()
    hd = _headers_digest()
    jobs = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, hd, force), srcs))
    out = ext_path()
    link_key = hashlib.sha256("".join(str(o) for o in objs).encode()).hexdigest()[:16]
    stamp = OBJ / "link.stamp"
    if out.exists() and stamp.exists() and stamp.read_text() == link_key and not force:
        return out
    tmp = out.with_suffix(".tmp.so")
    cmd = [hipcc(), "-shared", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(tmp),
           "-L/opt/rocm/lib", "-lhiprtc", "-Wl,-rpath,/opt/rocm/lib"]
    if _sanitize():
        cmd += [f"-fsanitize={_sanitize()}"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, out)
    stamp.write_text(link_key)
    if verbose:
        print(f"built {out}")
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--no-aot", action="store_true", help="skip the generated-kernel code objects")
    a = ap.parse_args(argv)
    build(force=a.force, jobs=a.jobs, verbose=True)
    if not a.no_aot:
        sys.path.insert(0, str(ROOT))
        from igloo_amd.ops import jit
        print("jit aot:", jit.aot_compile(jobs=a.jobs or 8))
    return 0


if __name__ == "__main__":
    sys.exit(main())
