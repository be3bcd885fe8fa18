"""Probe: are zero-fills (torch.zeros / zero_) inside a captured HIP graph
ordered correctly against the kernels around them on replay? A block is
written with 7s, freed, re-allocated as torch.zeros inside the same capture,
then summed; every replay must give 0. Also dumps the graph (DOT) so the node
kinds (kernel / memset / memcpy) are visible."""
import os
import re

import torch

dev = torch.device("cuda:0")
n = int(os.environ.get("N", str(1 << 22)))
s = torch.cuda.Stream()
g = torch.cuda.CUDAGraph()
g.enable_debug_mode()
torch.cuda.synchronize()
with torch.cuda.stream(s):
    g.capture_begin()
    a = torch.empty(n, dtype=torch.int64, device=dev).fill_(7)
    x = a.sum()
    del a
    b = torch.zeros(n, dtype=torch.int64, device=dev)      # may take a's block
    c = torch.empty(n, dtype=torch.int64, device=dev)
    c.zero_()
    out = torch.stack([b.sum(), c.sum(), x])
    g.capture_end()
torch.cuda.current_stream().wait_stream(s)
os.makedirs("gpurun_out", exist_ok=True)
try:
    g.debug_dump(os.path.abspath("gpurun_out/memset_probe.dot"))
    txt = open("gpurun_out/memset_probe.dot").read()
    print("node kinds:", sorted(set(re.findall(r"(MEMSET|MEMCPY|KERNEL|Memset|Memcpy|Kernel)", txt))), flush=True)
except OSError as e:
    print("no dump:", e, flush=True)
bad = 0
for i in range(200):
    g.replay()
    v = out.tolist()
    if v[0] != 0 or v[1] != 0 or v[2] != 7 * n:
        bad += 1
        if bad <= 5:
            print("replay", i, "got", v, flush=True)
print("bad replays:", bad, "of 200", flush=True)

# large reductions: torch's multi-block "global reduce" zeroes a semaphore
# buffer with a memset inside the reduction
big = torch.zeros(int(os.environ.get("NB", str(150_000_000))), dtype=torch.int64, device=dev)
g2 = torch.cuda.CUDAGraph()
torch.cuda.synchronize()
with torch.cuda.stream(s):
    g2.capture_begin()
    r1 = (big == 0).all()
    r2 = (big + 1).sum()
    r3 = big.min()
    g2.capture_end()
torch.cuda.current_stream().wait_stream(s)
bad = 0
for i in range(100):
    g2.replay()
    v = [bool(r1.item()), int(r2.item()), int(r3.item())]
    if v != [True, big.numel(), 0]:
        bad += 1
        if bad <= 5:
            print("reduce replay", i, "got", v, flush=True)
print("bad reduce replays:", bad, "of 100", flush=True)
