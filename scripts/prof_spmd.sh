set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/spo" -o run -- python3 scripts/spmd_overhead.py --sf ${SF:-10} --queries ${QS:-1-22} > gpurun_out/spmd_overhead_run.log 2>&1
rc=$?; echo "run rc=$rc"; tail -25 gpurun_out/spmd_overhead_run.log
[ $rc -eq 0 ] || exit $rc
T=$(find gpurun_out/spo -name "*kernel_trace.csv" | head -1)
python3 scripts/spmd_overhead.py --parse "$T" --queries ${QS:-1-22} --sf ${SF:-10} --top ${TOP:-12} --seq ${SEQ:-0} > gpurun_out/spmd_overhead.txt 2>&1
rm -rf gpurun_out/spo
head -60 gpurun_out/spmd_overhead.txt
