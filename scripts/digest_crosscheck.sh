# SF100 result digests of the default paths vs the paths named by IGLOO_DEBUG tokens (OLD, default: the
# partitioned aggregate and the mask tile counts switched off): bash scripts/digest_crosscheck.sh
cd /root/repo && export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --source hbm --sf 100 --steps 1 --warmup 1 --eager-steps 0 --vary-params 0 --digests-out gpurun_out/dig_new.json > gpurun_out/s39_a.log 2>&1 || exit $?
IGLOO_DEBUG=${OLD:-no_agg_part,no_mask_counts} timeout -k 10 400 python3 bench.py --source hbm --sf 100 --steps 1 --warmup 1 --eager-steps 0 --vary-params 0 --digests-out gpurun_out/dig_old.json > gpurun_out/s39_b.log 2>&1 || exit $?
python3 - <<'PY' > gpurun_out/s39_cmp.txt
import json
a = json.load(open("gpurun_out/dig_new.json")); b = json.load(open("gpurun_out/dig_old.json"))
same = [q for q in a if a[q] == b.get(q)]
print(f"{len(same)}/{len(a)} query digests equal between the new paths (partitioned aggregate, mask tile counts) and the old ones")
print("differ:", [q for q in a if a[q] != b.get(q)])
PY
cat gpurun_out/s39_cmp.txt
