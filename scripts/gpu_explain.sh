set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out && export TMPDIR=/tmp
IGLOO_LOG=debug timeout -k 10 400 python -u scripts/explain_compare.py --sf ${SF:-10} --queries ${QS:-10,21,2,17} > gpurun_out/explain_compare.log 2>&1
rc=$?; echo "explain rc=$rc"; grep -c "=====" gpurun_out/explain_compare.log
