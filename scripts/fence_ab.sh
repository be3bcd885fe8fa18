set -o pipefail
mkdir -p gpurun_out
for F in 0 1 0 1; do
  IGLOO_SEARCH_FENCE=$F timeout -k 10 300 python -u bench.py --source hbm --steps 10 --warmup 5 --per-query > gpurun_out/fence_ab_$F.log 2>&1 || exit $?
  echo "FENCE=$F $(tail -1 gpurun_out/fence_ab_$F.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["verified"])')"
done
