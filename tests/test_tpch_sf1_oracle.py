"""Independent oracle: the CPU engine against sqlite3 (its own parser, planner
and executor) on all 22 TPC-H queries (scripts/oracle_sf.py). The GPU suites
compare with the CPU engine (tests/test_tpch_sf1_gpu.py), so this anchors them.
SF0.1 runs in every default CPU test run (~1 minute); SF1 takes several
minutes and runs when IGLOO_SLOW=1 (committed run:
profiles/r3_oracle_sf1_cpu_vs_sqlite.log)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _oracle(sf: float, tmp_path):
    out = tmp_path / "oracle.json"
    p = subprocess.run([sys.executable, "scripts/oracle_sf.py", "--sf", str(sf), "--json", str(out)], cwd=ROOT,
                       capture_output=True, text=True, timeout=3600)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    res = json.loads(out.read_text())
    assert res["mismatched"] == [] and len(res["queries"]) == 22


def test_tpch_sf01_cpu_engine_matches_sqlite(tmp_path):
    _oracle(0.1, tmp_path)


@pytest.mark.slow
@pytest.mark.skipif(os.environ.get("IGLOO_SLOW") != "1", reason="slow: set IGLOO_SLOW=1")
def test_tpch_sf1_cpu_engine_matches_sqlite(tmp_path):
    _oracle(1.0, tmp_path)
