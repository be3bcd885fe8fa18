set -o pipefail
mkdir -p gpurun_out
for SPEC in 0 1; do
  IGLOO_SPMD_SPECULATE=$SPEC IGLOO_BENCH_SHARE_GPU=1 timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2953$SPEC bench.py --gpus 2 --sf 1 --steps 4 --warmup 2 > gpurun_out/bench_2rank_spec$SPEC.log 2>&1 || exit $?
  echo "SPMD_SPECULATE=$SPEC $(tail -1 gpurun_out/bench_2rank_spec$SPEC.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["verified"], d["speculation"])')"
done
