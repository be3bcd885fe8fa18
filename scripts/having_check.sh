set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_having_gpu.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/having_tests.log 2>&1
rc=$?; echo "having tests rc=$rc"; tail -3 gpurun_out/having_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --source hbm --queries 18 --steps 5 --warmup 3 --eager-steps 1 --vary-params 1 --per-query > gpurun_out/q18.log 2>&1
rc=$?; echo "q18 rc=$rc"; grep "Q18\|eager\|ad-hoc" gpurun_out/q18.log | tail -4; tail -1 gpurun_out/q18.log | cut -c1-150
