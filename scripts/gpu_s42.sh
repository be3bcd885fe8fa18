cd /root/repo && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_tpch_gpu.py > gpurun_out/s42_tests.log 2>&1 || exit $?
VAR=IGLOO_DEBUG VALS="pack_bits_scalar none pack_bits_scalar none" QS=3,5,7,9,10,18,21 bash scripts/ab_env.sh > gpurun_out/s42_ab.log 2>&1
