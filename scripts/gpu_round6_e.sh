# regex GPU tests again, then a kernel trace of the graphed SF10 suite (HBM tables) with gap analysis
cd /root/repo && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_sql_datafusion_surface.py -m gpu -k "regex or similar" > gpurun_out/r6_gpu_regex.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/r6_gpu_regex.log
[ $rc -le 1 ] || exit $rc
IGLOO_PROF_GAP=1 timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6_trace_sf10 -o run -- python3 bench.py --source hbm --sf 10 --steps 5 --warmup 4 --eager-steps 0 --vary-params 0 > gpurun_out/r6_trace_sf10.log 2>&1 || exit $?
f=$(find gpurun_out/r6_trace_sf10 -name "*kernel_trace.csv" | head -1)
python3 scripts/kernel_summary.py "$f" --steps 5 --top 60 > gpurun_out/r6_kernel_summary_sf10.txt
rm -f "$f"
exit $rc
