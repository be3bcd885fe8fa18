timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_sql_datafusion_surface.py -m gpu > gpurun_out/r6_gpu_surface.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/r6_gpu_surface.log
if [ $rc -le 1 ]; then IGLOO_CHECK_KEY_TAGS=1 timeout -k 10 300 python -u scripts/dbg_spmd_query.py 9 4 0 '[["tags",{"IGLOO_CHECK_KEY_TAGS":"1"},[]]]' > gpurun_out/r6_dbg_q9_tags.log 2>&1; fi
exit $rc
