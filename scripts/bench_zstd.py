"""Throughput of the GPU ZSTD page decoder (csrc/kernels/zstd.hip) on
Parquet-page-sized frames: --pages frames of --page-kb uncompressed bytes of
one data kind (TPC-H-like text, sorted int64 keys, small ints, doubles),
compressed by pyarrow's libzstd, decoded in one pq_zstd launch; output
checked against the input.   python scripts/bench_zstd.py [--kind text]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import numpy as np  # noqa: E402
import pyarrow as pa  # noqa: E402
import torch  # noqa: E402

from igloo_amd.ops._lib import native, ptr  # noqa: E402


def page(kind, nbytes, rng, i):
    if kind == "text":
        words = ["special", "requests", "carefully", "final", "deposits", "the", "of", "ironic", "pinto", "beans",
                 "furiously", "slyly", "regular", "accounts", "blithely", "quick"]
        s = " ".join(rng.choice(words, nbytes // 6)).encode()
        return s[:nbytes]
    if kind == "keys":
        n = nbytes // 8
        return (np.repeat(np.arange(i * n // 4, i * n // 4 + n // 4 + 1, dtype=np.int64), 4)[:n]).tobytes()
    if kind == "smallint":
        return rng.integers(1, 51, nbytes // 4).astype(np.int32).tobytes()
    return rng.normal(size=nbytes // 8).round(2).tobytes()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", default="text", choices=["text", "keys", "smallint", "doubles"])
    ap.add_argument("--pages", type=int, default=2048)
    ap.add_argument("--page-kb", type=int, default=128)
    ap.add_argument("--level", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    N = native()
    rng = np.random.default_rng(0)
    codec = pa.Codec("zstd", compression_level=a.level)
    raws = [page(a.kind, a.page_kb << 10, rng, i) for i in range(min(a.pages, 64))]
    raws = [raws[i % len(raws)] for i in range(a.pages)]
    comps = [codec.compress(r, asbytes=True) for r in raws]
    src_off = np.cumsum([0] + [len(c) for c in comps[:-1]])
    dst_off = np.cumsum([0] + [(len(r) + 15) // 16 * 16 for r in raws[:-1]])
    jobs = np.zeros(a.pages, dtype=[("src", "<i8"), ("dst", "<i8"), ("slen", "<i4"), ("dlen", "<i4"),
                                     ("codec", "<i4"), ("pad", "<i4")])
    jobs["src"], jobs["dst"] = src_off, dst_off
    jobs["slen"], jobs["dlen"] = [len(c) for c in comps], [len(r) for r in raws]
    jobs["codec"] = 6
    dev = "cuda"
    raw = torch.frombuffer(bytearray(b"".join(comps) + bytes(64)), dtype=torch.uint8).to(dev)
    jt = torch.frombuffer(bytearray(jobs.tobytes()), dtype=torch.uint8).to(dev)
    out_bytes = int(dst_off[-1]) + len(raws[-1])
    dec = torch.zeros(out_bytes + 64, dtype=torch.uint8, device=dev)
    slots = N.pq_zstd_slots(a.pages)
    lit = torch.empty(slots << 17, dtype=torch.uint8, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    N.pq_zstd(ptr(jt), a.pages, ptr(raw), ptr(dec), ptr(lit), slots, ptr(err), s)
    torch.cuda.synchronize()
    assert int(err.item()) == 0, int(err.item())
    host = dec.cpu().numpy().tobytes()
    for i in (0, a.pages // 2, a.pages - 1):
        assert host[dst_off[i]:dst_off[i] + len(raws[i])] == raws[i], i
    t = time.perf_counter()
    for _ in range(a.reps):
        N.pq_zstd(ptr(jt), a.pages, ptr(raw), ptr(dec), ptr(lit), slots, ptr(err), s)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / a.reps
    comp_b = sum(len(c) for c in comps)
    raw_b = sum(len(r) for r in raws)
    print(f"kind={a.kind} pages={a.pages} page={a.page_kb}KiB level={a.level} ratio={raw_b / comp_b:.2f} "
          f"{dt * 1e3:.2f} ms  in {comp_b / dt / 1e9:.2f} GB/s  out {raw_b / dt / 1e9:.2f} GB/s", flush=True)


if __name__ == "__main__":
    main()
