#!/usr/bin/env bash
# Host sanitizer run: the SQL parser and the Parquet Thrift
# decoders built with -fsanitize=address,undefined and driven over the TPC-H
# queries, the reference-compat SQL and a few generated Parquet files, each
# truncated and byte-flipped (csrc/tools/fuzz_host.cpp). CPU only.
set -euo pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
OUT="${OUT:-/tmp/igloo_sanitize}"
mkdir -p "$OUT"
CXX=/opt/rocm/lib/llvm/bin/clang++
$CXX -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined \
  -D__HIP_PLATFORM_AMD__ -I"$R/csrc" -I/opt/rocm/include \
  "$R/csrc/tools/fuzz_host.cpp" "$R/csrc/sql/parser.cpp" "$R/csrc/io/parquet_meta.cpp" \
  -lpthread -o "$OUT/fuzz_host"
python3 - "$OUT" <<'PY'
import os, sys
sys.path.insert(0, os.environ.get("R", "."))
out = sys.argv[1]
from igloo_amd.models.tpch import queries
import pyarrow as pa, pyarrow.parquet as pq
extra = ["SELECT 42 AS answer", "SELECT name, age FROM users WHERE age > 30 ORDER BY age NULLS FIRST LIMIT 5",
         "SELECT capitalize(name) FROM t", "CREATE EXTERNAL TABLE t STORED AS PARQUET LOCATION '/x'",
         "SELECT a, sum(b) FILTER (WHERE c) FROM t GROUP BY ROLLUP (a)", "EXPLAIN ANALYZE SELECT 1",
         "SELECT CASE WHEN x IN (1,2) THEN 'a' ELSE NULL END, CAST(y AS DECIMAL(15,2)) FROM t"]
with open(os.path.join(out, "corpus.sql"), "w") as f:
    for q in list(queries.QUERIES.values()) + extra:
        f.write(q.strip() + "\n\n")
t = pa.table({"k": pa.array(range(1000), pa.int64()), "s": pa.array([f"v{i % 13}" for i in range(1000)]),
              "d": pa.array([i * 0.5 for i in range(1000)])})
for comp in ("snappy", "none"):
    pq.write_table(t, os.path.join(out, f"t_{comp}.parquet"), compression=comp, row_group_size=300)
PY
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  "$OUT/fuzz_host" "$OUT/corpus.sql" "$OUT"/t_*.parquet
