"""Host sanitizer run: SQL parser + Parquet Thrift decoders under
AddressSanitizer / UBSan over a mutated corpus (scripts/sanitize_host.sh,
csrc/tools/fuzz_host.cpp). GPU ASan is not available on the pool; this covers
the native code that parses untrusted input."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not os.path.exists("/opt/rocm/lib/llvm/bin/clang++"), reason="no clang")
def test_parser_and_parquet_decoders_sanitizer_clean(tmp_path):
    env = dict(os.environ, R=ROOT, OUT=str(tmp_path))
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "sanitize_host.sh")], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "no sanitizer reports" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
