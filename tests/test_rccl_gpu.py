"""RCCL on the GPU box (one GPU: a world of one rank, ``force_spmd``).

* every collective parallel/comm.py issues runs through the nccl (= RCCL)
  backend — all_to_all_single, all_gather_into_tensor, batch_isend_irecv,
  all_reduce, broadcast — bypassing the world-of-one short-circuit;
* the same collectives captured inside a HIP graph replay correctly (the SPMD
  query graphs of engine.py capture exchanges this way);
* all 22 TPC-H queries run through the SPMD path (every exchange real) over
  RCCL, with replayed readbacks and query graphs, and match a single-rank
  engine (scripts/spmd_world1.py).

Each case runs in a fresh subprocess (its own process group)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_API = r'''
import os, sys, torch
import torch.distributed as dist
sys.path.insert(0, os.environ["ROOT"])
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ["PORT"], RANK="0", WORLD_SIZE="1")
from igloo_amd.parallel.comm import Communicator
dev = torch.device("cuda:0")
c = Communicator.init(backend="nccl", device=dev, force_spmd=True, timeout_s=120)
assert c.backend == "nccl" and c.spmd and c.world_size == 1
x = torch.arange(1000, dtype=torch.int64, device=dev)
y, rc = c.all_to_all_v(x, [1000])                      # all_to_all_single
assert rc == [1000] and torch.equal(y, x)
assert c.all_to_all_counts([7]) == [7]
g, cnt = c.all_gather_v(x[:300], [300])                 # all_gather_into_tensor
assert cnt == [300] and torch.equal(g, x[:300])
assert c.allgather_ints([3, 4]) == [[3, 4]]
assert c.allreduce_ints([5, 6]) == [5, 6]               # all_reduce
t = c.allreduce_tensor(torch.tensor([1.5, 2.5], dtype=torch.float64, device=dev), "max")
assert t.tolist() == [1.5, 2.5]
b = c.broadcast_tensor(torch.full((4,), 9, dtype=torch.int32, device=dev))   # broadcast
assert b.tolist() == [9] * 4
# point-to-point (the uneven all-gather-v path): send to / receive from self
r = torch.empty(200, dtype=torch.int64, device=dev)
for q in dist.batch_isend_irecv([dist.P2POp(dist.isend, x[:200], 0), dist.P2POp(dist.irecv, r, 0)]):
    q.wait()
assert torch.equal(r, x[:200])
# collectives inside a captured HIP graph, replayed with new inputs
src = torch.zeros(512, dtype=torch.int64, device=dev)
dst = torch.empty_like(src)
red = torch.zeros(8, dtype=torch.int64, device=dev)
s = torch.cuda.Stream(dev)
s.wait_stream(torch.cuda.current_stream(dev))
with torch.cuda.stream(s):
    dist.all_to_all_single(dst, src * 2, [512], [512]); dist.all_reduce(red)   # warm the communicator
torch.cuda.current_stream(dev).wait_stream(s)
torch.cuda.synchronize()
gr = torch.cuda.CUDAGraph()
with torch.cuda.graph(gr):
    tmp = src * 2
    dist.all_to_all_single(dst, tmp, [512], [512])
    dist.all_reduce(red)
    ag = torch.empty(512, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(ag, dst)
for k in (1, 5):
    src.copy_(torch.arange(512, device=dev) + k)
    red.fill_(k)
    gr.replay()
    torch.cuda.synchronize()
    assert torch.equal(dst, (torch.arange(512, device=dev) + k) * 2), k
    assert torch.equal(ag, dst) and red.tolist() == [k] * 8, k
c.shutdown()
print("RCCL_API_OK")
'''


def _port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return str(p)


def _run(args, timeout):
    env = dict(os.environ, ROOT=ROOT, PORT=_port(), MASTER_ADDR="127.0.0.1", MASTER_PORT=_port())
    return subprocess.run(args, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)


def test_rccl_world1_every_collective_and_graph_capture():
    p = _run([sys.executable, "-c", _API], 240)
    assert p.returncode == 0 and "RCCL_API_OK" in p.stdout, p.stdout[-3000:] + p.stderr[-3000:]


def test_tpch_spmd_path_over_rccl_with_graphs(tmp_path):
    out = tmp_path / "spmd.json"
    p = _run([sys.executable, "scripts/spmd_world1.py", "--sf", "0.05", "--device", "cuda:0", "--backend", "nccl",
              "--runs", "6", "--json", str(out)], 600)
    assert p.returncode == 0, p.stdout[-4000:] + p.stderr[-4000:]
    res = json.loads(out.read_text())
    print({k: v for k, v in res.items() if k != "queries"})
    assert not res["mismatches"]
    modes = {q: [r["mode"] for r in rs] for q, rs in res["queries"].items()}
    graphed = [q for q, m in modes.items() if m[-1] == "graph"]
    assert res["graphs"]["failed"] == 0 and res["graphs"]["mismatch"] == 0, res["graphs"]
    assert len(graphed) >= 11, (graphed, res["graph_errors"])
