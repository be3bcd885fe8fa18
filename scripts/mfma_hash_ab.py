"""MFMA vs VALU for the two hash / compare shapes of the north star
(csrc/kernels/mfma_probe.hip), on data of the TPC-H shapes they serve:

(a) composite-key hash of four int32 key columns, 60M rows (SF10 lineitem
    size: Q9's (partkey, suppkey, orderkey, linenumber)-like keys);
(b) IN-list compare of c_phone-like strings' first 2 bytes against 7
    patterns (Q22's country codes) and of 10-byte p_type-like strings
    against 16 patterns, 15M rows.

Each variant is checked against the other (hash: against a host replay of
the same MFMA projection is not needed -- the two hashes differ by design,
so the check is the hash's collision rate on distinct keys; IN-list: equal
masks), then timed (median of 20 launches). Run under rocprofv3 --pmc for
SQ_INSTS_MFMA / SQ_INSTS_VALU / FETCH_SIZE (scripts/mfma_hash_ab.sh)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=60_000_000)
    ap.add_argument("--str-rows", type=int, default=15_000_000)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    import numpy as np
    import torch
    from igloo_amd.ops._lib import native, ptr
    N = native()
    dev = "cuda:0"
    s = torch.cuda.current_stream().cuda_stream
    out = {}

    def timeit(fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        return float(np.median(ts))

    if a.only in ("", "hash"):
        n = a.rows
        g = torch.Generator(device=dev).manual_seed(1)
        ks = [torch.randint(0, 2**31 - 1, (n,), dtype=torch.int32, device=dev, generator=g) for _ in range(4)]
        proj = torch.randint(-127, 128, (16, 16), dtype=torch.int8, generator=torch.Generator().manual_seed(7)).to(dev)
        res = {}
        for mf in (False, True):
            o = torch.empty(n, dtype=torch.uint32, device=dev) if hasattr(torch, "uint32") else \
                torch.empty(n, dtype=torch.int32, device=dev)
            ms = timeit(lambda: N.probe_hash16(mf, ptr(ks[0]), ptr(ks[1]), ptr(ks[2]), ptr(ks[3]), n, ptr(proj),
                                               ptr(o), s))
            h = o.view(torch.int32).to(torch.int64)
            distinct = torch.unique(h[: 1 << 22]).numel()
            res["mfma" if mf else "valu"] = {"ms": round(ms, 4), "gb_s": round(n * 20 / ms / 1e6, 1),
                                             "distinct_of_4M": distinct}
        out["hash16"] = res
    if a.only in ("", "inlist"):
        n = a.str_rows
        rng = np.random.default_rng(3)
        # Q22: substring(c_phone, 1, 2) IN (7 codes) -- the 2-byte prefixes as strings;
        # p_type-like 10-byte strings against 16 values
        for name, length, npat, alphabet in (("phone_cc2", 2, 7, b"0123456789"), ("type10", 10, 16, b"ABCD")):
            body = rng.choice(np.frombuffer(alphabet, np.uint8), size=(n, length))
            chars = torch.from_numpy(body.reshape(-1).copy()).to(dev)
            off = torch.arange(n + 1, dtype=torch.int64, device=dev) * length
            pats = [bytes(body[i]) for i in rng.choice(n, npat, replace=False)]
            blob = b"".join(p.ljust(16, b"\0") for p in pats)
            res, masks = {}, {}
            for mf in (False, True):
                o = torch.empty(n, dtype=torch.uint8, device=dev)
                ms = timeit(lambda: N.probe_inlist16(mf, ptr(off), ptr(chars), n, blob, npat, length, ptr(o), s))
                masks[mf] = o.clone()
                res["mfma" if mf else "valu"] = {"ms": round(ms, 4), "gb_s": round((n * (length + 8)) / ms / 1e6, 1),
                                                 "hits": int(o.sum().item())}
            want = np.isin(np.frombuffer(body.tobytes(), dtype=f"S{length}"), np.array(pats, dtype=f"S{length}"))
            res["valu_matches_numpy"] = bool(np.array_equal(masks[False].cpu().numpy().astype(bool), want))
            res["masks_equal"] = bool(torch.equal(masks[False], masks[True]))
            out[f"inlist_{name}"] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
