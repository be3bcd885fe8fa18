#!/bin/bash
# 2-rank (shared GPU, gloo) SF1 bench per env configuration: verification and
# speculation counts — rehearsal of the multi-GPU path on a one-GPU box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
i=0
for cfg in "${@:-IGLOO_NONE=1}"; do
  i=$((i+1))
  env IGLOO_BENCH_SHARE_GPU=1 $cfg timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NP:-2} \
    --master-addr 127.0.0.1 --master-port $((29540 + i)) bench.py --gpus ${NP:-2} --sf ${SF:-1} --steps 3 --warmup 1 \
    > gpurun_out/dist$i.log 2>&1 || { echo "$cfg failed"; tail -5 gpurun_out/dist$i.log; exit 1; }
  echo "== $cfg $(grep -o '"value": [0-9.]*' gpurun_out/dist$i.log) $(grep -o '"verified": [a-z]*' gpurun_out/dist$i.log) $(grep -o '"speculation": {[^}]*}' gpurun_out/dist$i.log) $(grep -c 'did not match' gpurun_out/dist$i.log) $(grep 'digests differ' gpurun_out/dist$i.log)"
done
