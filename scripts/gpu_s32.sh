cd /root/repo && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_gpu.py tests/test_jit_codegen.py tests/test_tpch_gpu.py > gpurun_out/s32_tests.log 2>&1 || exit $?
VAR=IGLOO_DEBUG VALS="no_mask_counts none no_mask_counts none" bash scripts/ab_env.sh > gpurun_out/s32_ab.log 2>&1
