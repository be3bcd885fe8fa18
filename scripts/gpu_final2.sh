set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_determinism_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_det.log 2>&1
rc=$?
echo "det exit $rc"; tail -3 gpurun_out/pytest_det.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_prof_graphs.sh
