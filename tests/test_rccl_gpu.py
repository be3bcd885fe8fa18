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
    p = _run([sys.executable, "-u", "scripts/rccl_probe.py"], 150)
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
