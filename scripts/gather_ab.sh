set -o pipefail
mkdir -p gpurun_out
for R in 4 8 4 8; do
  IGLOO_GATHER_ROWS=$R timeout -k 10 300 python -u bench.py --source hbm --steps 10 --warmup 5 > gpurun_out/gather_ab_$R.log 2>&1 || exit $?
  echo "R=$R $(tail -1 gpurun_out/gather_ab_$R.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["verified"])')"
done
