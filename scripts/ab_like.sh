set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "like" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/like_tests.log 2>&1
rc=$?; echo "like tests rc=$rc"; tail -2 gpurun_out/like_tests.log; [ $rc -eq 0 ] || exit $rc
for w in 0 1; do
  IGLOO_LIKE_WAVE=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ablike$w -o run -- python3 bench.py --source hbm --queries 13,16 --steps 3 --warmup 3 --eager-steps 0 --vary-params 0 --per-query > gpurun_out/ablike$w.log 2>&1
  rc=$?; echo "like wave=$w rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep "Q13\|Q16" gpurun_out/ablike$w.log
  f=$(find gpurun_out/ablike$w -name "*kernel_stats.csv" | head -1); grep -i "like" $f | cut -c1-200
  rm -f $(find gpurun_out/ablike$w -name "*kernel_trace.csv")
done
