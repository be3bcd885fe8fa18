# kernel trace of the graphed SF100 suite (HBM tables) listing every dispatch of
# the kernels matching $MATCH (duration, grid) -> gpurun_out/trace_dispatches.txt
cd /root/repo && export TMPDIR=/tmp
out=gpurun_out
IGLOO_PROF_GAP=1 timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $out/td_trace -o run -- \
    python3 bench.py --source hbm --steps 1 --warmup 4 --eager-steps 0 --vary-params 0 > $out/td_trace.log 2>&1 || exit $?
f=$(find $out/td_trace -name "*kernel_trace.csv" | head -1)
python3 scripts/kernel_summary.py "$f" --steps 1 --top 40 --dispatches "${MATCH:-probe_hits|probe_write|agg_global}" > $out/trace_dispatches.txt
rm -rf $out/td_trace
