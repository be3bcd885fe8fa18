cd /root/repo && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_join_paths_gpu.py > gpurun_out/s40_tests.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --source hbm --sf 100 --steps 10 --warmup 3 --eager-steps 0 --vary-params 0 --per-query > gpurun_out/s40_bench.log 2>&1
QS_T=5 bash scripts/gpu_s37.sh
