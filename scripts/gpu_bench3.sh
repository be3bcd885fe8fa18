set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --steps 8 --warmup 1 --per-query > gpurun_out/bench_sf100.log 2>&1
rc=$?
echo "exit $rc"
grep -E "cold suite|warmup|step|modes" gpurun_out/bench_sf100.log | cut -c1-300
exit $rc
