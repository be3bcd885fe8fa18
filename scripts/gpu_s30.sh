cd /root/repo && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_agg_partitioned_gpu.py > gpurun_out/s30_tests.log 2>&1 || exit $?
VAR=IGLOO_DEBUG VALS="no_agg_part none no_agg_part none" bash scripts/ab_env.sh > gpurun_out/s30_ab.log 2>&1
