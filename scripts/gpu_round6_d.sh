timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_sql_datafusion_surface.py -m gpu > gpurun_out/r6_gpu_surface.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/r6_gpu_surface.log
if [ $rc -le 1 ]; then
  for v in UNIQUE_PAIRS_SORTED UNIQUE_PAIRS_DENSE UNIQUE_PAIRS_TWO_KEY; do
    DBG_SET="igloo_amd.exec.joins.$v=0" timeout -k 10 120 python -u scripts/dbg_spmd_query.py 9 4 0 "[[\"no_$v\",{},[]]]" >> gpurun_out/r6_dbg_q9_split.log 2>&1 || exit 3
  done
  timeout -k 10 300 python -u scripts/prof_host_floor.py --sf 1 --suites 10 > gpurun_out/r6_prof_host_floor_sf1.log 2>&1 || exit 4
fi
exit $rc
