set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u bench.py --sf 1 --steps 5 --warmup 1 --per-query > gpurun_out/bench_sf1.log 2>&1 && \
timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 --per-query > gpurun_out/bench_sf100.log 2>&1
rc=$?
echo "exit $rc"
grep -E "cold suite|warmup|step" gpurun_out/bench_sf1.log | tr '\n' ' '; echo
tail -1 gpurun_out/bench_sf1.log | cut -c1-200; echo
grep -E "cold suite|warmup|step" gpurun_out/bench_sf100.log | tr '\n' ' '; echo
tail -1 gpurun_out/bench_sf100.log | cut -c1-200
exit $rc
