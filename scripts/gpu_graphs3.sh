set -o pipefail
mkdir -p gpurun_out
QS=16,20,21,22,2,1,3,4,5,6,7,8,9,10,11,12,13,14,15,17,18,19 timeout -k 10 300 python -u scripts/graph_debug.py > gpurun_out/graph_debug.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "exit $rc"; grep -E "run 5|volatile|abort" gpurun_out/graph_debug.log | sort | uniq -c | head -40; tail -3 gpurun_out/pytest_gpu.log
exit $rc
