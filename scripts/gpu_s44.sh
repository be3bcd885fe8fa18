cd /root/repo && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_agg_partitioned_gpu.py tests/test_kernels_gpu.py tests/test_tpch_gpu.py tests/test_fused_gpu.py tests/test_having_gpu.py > gpurun_out/s44_tests.log 2>&1 || exit $?
IGLOO_PROF_GAP=1 timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s44_trace -o run -- python3 bench.py --source hbm --steps 3 --warmup 4 --eager-steps 0 --vary-params 0 > gpurun_out/s44_trace.log 2>&1 || exit $?
python3 scripts/kernel_summary.py $(find gpurun_out/s44_trace -name "*kernel_trace.csv" | head -1) --steps 3 --top 70 > gpurun_out/s44_summary.txt
rm -rf gpurun_out/s44_trace
