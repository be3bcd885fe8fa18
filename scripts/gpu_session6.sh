# graph-captured result packing: graph / replay-safety / rccl tests, then the driver-config bench and a trace
cd /root/repo && export TMPDIR=/tmp
out=gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "graph or replay or rccl or tpch or spmd or bench" > $out/s6_pytest.log 2>&1 || exit $?
timeout -k 10 900 python3 -u bench.py --steps 20 --warmup 5 --per-query > $out/s6_bench_sf100.log 2>&1 || exit $?
IGLOO_PROF_GAP=1 timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $out/s6_trace -o run -- \
    python3 bench.py --source hbm --steps 3 --warmup 4 --eager-steps 0 --vary-params 0 > $out/s6_trace.log 2>&1 || exit $?
f=$(find $out/s6_trace -name "*kernel_trace.csv" | head -1)
python3 scripts/kernel_summary.py "$f" --steps 3 --top 70 > $out/s6_kernel_summary_sf100.txt
rm -rf $out/s6_trace
