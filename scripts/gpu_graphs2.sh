set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_sort_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_sort.log 2>&1 && \
QS=16,20,21,22,2,1,3,5,9 timeout -k 10 300 python -u scripts/graph_debug.py > gpurun_out/graph_debug.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_graphs_gpu.py tests/test_speculation_gpu.py -x -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_graphs.log 2>&1
rc=$?
echo "exit $rc"; tail -2 gpurun_out/pytest_sort.log; grep -E "run 5|volatile|abort" gpurun_out/graph_debug.log | sort | uniq -c | head -30; tail -3 gpurun_out/pytest_graphs.log
exit $rc
