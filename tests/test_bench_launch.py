"""bench.py's multi-rank contract: ``--gpus N`` launches N real ranks itself
(no external torchrun), reports the world every rank saw, and refuses a world
it cannot build (more ranks than GPUs, or a launcher world != --gpus)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None, timeout=600):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.pop("RANK", None)
    e.pop("LOCAL_RANK", None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          env=e, timeout=timeout, cwd=ROOT)


def test_bench_self_launches_n_ranks(tmp_path):
    p = _run(["--cpu", "--gpus", "4", "--sf", "0.01", "--steps", "1", "--warmup", "0", "--eager-steps", "0",
              "--vary-params", "0", "--data-dir", str(tmp_path)])
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout          # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 4 and d["world"] == 4 and d["verified"] is True
    assert d["config"]["parallelism"] == "dp4"
    assert sorted(r["rank"] for r in d["ranks"]) == [0, 1, 2, 3]
    assert all(r["world"] == 4 and r["collectives"] > 0 for r in d["ranks"])
    assert abs(d["value"] - max(r["timed_region_s"] for r in d["ranks"]) / d["steps"]) < 2e-3


def test_bench_refuses_more_ranks_than_gpus():
    # this container has no GPU: --gpus 2 without --cpu cannot place 2 ranks
    p = _run(["--gpus", "2", "--sf", "0.01"], timeout=300)
    assert p.returncode == 2, (p.returncode, p.stderr[-2000:])
    assert "GPU" in p.stderr


def test_bench_refuses_world_mismatch():
    p = _run(["--cpu", "--gpus", "2", "--sf", "0.01"], env={"WORLD_SIZE": "3", "RANK": "0"}, timeout=300)
    assert p.returncode == 2 and "WORLD_SIZE=3" in p.stderr, p.stderr[-2000:]
