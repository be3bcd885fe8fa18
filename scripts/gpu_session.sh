# One GPU session: the GPU test suite, the driver-config bench (SF100
# Parquet) and a kernel trace of the graphed SF100 suite with gap pairs.
# Every step under its own time limit; the first failing step ends it.
cd /root/repo && export TMPDIR=/tmp
out=gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $out/s_pytest_gpu.log 2>&1 || exit $?
timeout -k 10 900 python3 -u bench.py --steps 20 --warmup 5 --per-query > $out/s_bench_sf100.log 2>&1 || exit $?
IGLOO_PROF_GAP=1 timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $out/s_trace_sf100 -o run -- \
    python3 bench.py --source hbm --steps 3 --warmup 4 --eager-steps 0 --vary-params 0 > $out/s_trace_sf100.log 2>&1 || exit $?
f=$(find $out/s_trace_sf100 -name "*kernel_trace.csv" | head -1)
python3 scripts/kernel_summary.py "$f" --steps 3 --top 70 > $out/s_kernel_summary_sf100.txt
rm -rf $out/s_trace_sf100
