# Kernel trace of single queries of the graphed SF100 suite (HBM tables), every dispatch listed:
#   QS_T="5 13" bash scripts/gpu_query_trace.sh -> gpurun_out/q<N>_dispatches.txt
cd /root/repo && export TMPDIR=/tmp
for q in ${QS_T:-5}; do
IGLOO_PROF_GAP=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/qt$q -o run -- python3 bench.py --source hbm --queries $q --steps 2 --warmup 3 --eager-steps 0 --vary-params 0 > gpurun_out/qt$q.log 2>&1 || exit $?
python3 scripts/kernel_summary.py $(find gpurun_out/qt$q -name "*kernel_trace.csv" | head -1) --steps 2 --top 25 --dispatches "." > gpurun_out/q${q}_dispatches.txt
rm -rf gpurun_out/qt$q
done
