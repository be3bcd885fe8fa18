set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_graphs_gpu.py tests/test_join_paths_gpu.py tests/test_tpch_gpu.py tests/test_tpch_sf1_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_part.log 2>&1 && \
timeout -k 10 600 python -u bench.py --steps 8 --warmup 5 --per-query > gpurun_out/bench_sf100.log 2>&1
rc=$?
echo "exit $rc"
tail -2 gpurun_out/pytest_part.log
grep -E "cold suite|warmup|step|modes|graphs:|not captured" gpurun_out/bench_sf100.log | cut -c1-400 | sort | uniq -c | sort -rn | head -30
exit $rc
IGLOO_BENCH_SHARE_GPU=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --sf 1 --steps 2 --warmup 1 > gpurun_out/bench_2rank.log 2>&1
echo "2-rank exit $?"; tail -1 gpurun_out/bench_2rank.log | cut -c1-300
