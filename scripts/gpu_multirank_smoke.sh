set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
IGLOO_BENCH_SHARE_GPU=1 timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --sf 1 --steps 2 --warmup 1 > gpurun_out/bench_2rank.log 2>&1
rc=$?
echo "exit $rc"; tail -2 gpurun_out/smoke.log; tail -1 gpurun_out/bench_2rank.log | cut -c1-400
exit $rc
