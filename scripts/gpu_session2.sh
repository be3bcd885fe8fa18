# sort kernels (one-workgroup rewrite), a SF100 kernel trace with gap pairs,
# the per-query host floor at SF1, the 10M-row window query's kernels
cd /root/repo && export TMPDIR=/tmp
out=gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_sort_gpu.py -p no:cacheprovider > $out/s2_sort.log 2>&1 || exit $?
IGLOO_PROF_GAP=1 timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $out/s2_trace -o run -- \
    python3 bench.py --source hbm --steps 3 --warmup 4 --eager-steps 0 --vary-params 0 > $out/s2_trace.log 2>&1 || exit $?
f=$(find $out/s2_trace -name "*kernel_trace.csv" | head -1)
python3 scripts/kernel_summary.py "$f" --steps 3 --top 70 > $out/s2_kernel_summary_sf100.txt
rm -rf $out/s2_trace
timeout -k 10 300 python3 -u scripts/prof_host_floor.py --sf 1 --suites 10 > $out/s2_host_floor_sf1.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/s2_win -o run -- \
    python3 -m pytest -x -q tests/test_window_wide_gpu.py -k sliding -p no:cacheprovider > $out/s2_window.log 2>&1
f=$(find $out/s2_win -name "*kernel_stats.csv" | head -1); cp "$f" $out/s2_window_kernel_stats.csv; rm -rf $out/s2_win
