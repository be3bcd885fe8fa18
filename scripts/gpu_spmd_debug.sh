set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
IGLOO_LOG=debug timeout -k 10 300 python -u scripts/spmd_world1.py --sf 1 --device cuda:0 --backend nccl --runs 4 --queries ${QS:-1,10,22} > gpurun_out/spmd_debug.log 2>&1
rc=$?; echo "spmd debug rc=$rc"; grep -c "igloo" gpurun_out/spmd_debug.log; tail -2 gpurun_out/spmd_debug.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
bash scripts/prof_spmd.sh
