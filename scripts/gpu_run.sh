#!/bin/bash
# One GPU session on the gpurun box, by mode (several may be given, run in
# order). Every GPU step has its own time limit and the script stops at the
# first failing step; logs and summaries land in gpurun_out/.
#
#   tests   pytest -m gpu (the driver's round-end GPU tier)
#   bench   bench.py at the driver's SF100 configuration (--steps 20 --warmup 5)
#   spmd    multi-GPU code path on one GPU: scripts/spmd_world1.py (SF0.5, RCCL,
#           every collective real) + bench.py with IGLOO_FORCE_SPMD=1 at SF100
#   prof    rocprofv3 kernel trace of the warm SF100 suite (query graphs);
#           per-kernel summary of the timed steps (scripts/kernel_summary.py)
#   profq   per-query kernel summaries (QS="9 10 13" query sets, HBM tables)
#   jitcache  compile the suite's generated kernels at SF100 (validation
#           parameters only: ad-hoc runs must not find theirs precompiled) into
#           gpurun_out/jit_cache
#   jitsources  record generated-kernel sources (igloo_amd/jit_sources)
#   proj    per-query 8-GPU projection (scripts/spmd_projection.py) at SF100
#   rbsites blocking readbacks per query, parameter-dependent or not
#   pmc     rocprofv3 counter passes (FETCH_SIZE / WRITE_SIZE / instruction
#           mix; one pass per counter set, --kernel-trace only) over the warm
#           graphed suite; per-kernel bandwidth table (scripts/pmc_summary.py)
#
#   gpurun -- 'bash scripts/gpu_run.sh tests bench'
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
for mode in "$@"; do
  case "$mode" in
    tests)
      timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
        -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
      rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/pytest_gpu.log ;;
    bench)
      timeout -k 10 1000 python -u bench.py --steps 20 --warmup 5 --per-query > gpurun_out/bench_sf100.log 2>&1
      rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_sf100.log | cut -c1-400 ;;
    spmd)
      timeout -k 10 300 python -u scripts/spmd_world1.py --sf 0.5 --device cuda:0 --backend nccl --runs 6 \
        --json gpurun_out/spmd_sf05.json > gpurun_out/spmd_sf05.log 2>&1
      rc=$?; echo "spmd_world1 rc=$rc"; tail -1 gpurun_out/spmd_sf05.log | cut -c1-300
      [ $rc -eq 0 ] || exit $rc
      IGLOO_FORCE_SPMD=1 timeout -k 10 900 python -u bench.py --steps 10 --warmup 5 --per-query \
        > gpurun_out/bench_sf100_spmd1.log 2>&1
      rc=$?; echo "spmd bench rc=$rc"; tail -1 gpurun_out/bench_sf100_spmd1.log | cut -c1-400 ;;
    prof)
      IGLOO_PROF_GAP=1 timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" --steps 3 --warmup 5 --eager-steps 0 \
        --vary-params 0 > gpurun_out/prof.log 2>&1
      rc=$?; echo "prof rc=$rc"
      if [ $rc -eq 0 ]; then
        T=$(find gpurun_out/prof -name "*kernel_trace.csv" | head -1)
        python3 scripts/kernel_summary.py "$T" --steps 3 --top 40 > gpurun_out/kernel_summary.txt
        python3 scripts/aten_share.py "$T" --steps 3 > gpurun_out/aten_share.txt
        head -12 gpurun_out/kernel_summary.txt; rm -f "$T"
      fi ;;
    pmc)
      i=0
      while read -r SET; do
        [ -z "$SET" ] && continue
        i=$((i+1))
        IGLOO_PROF_GAP=1 timeout -s KILL 600 rocprofv3 --kernel-trace --pmc $SET --output-format csv \
          -d "$R/gpurun_out/pmc/p$i" -o run -- python3 "$R/bench.py" --source hbm --sf ${SF:-100} --steps 1 \
          --warmup 5 --eager-steps 0 --vary-params 0 > gpurun_out/pmc_p$i.log 2>&1
        rc=$?; echo "pmc pass $i ($SET) rc=$rc"; [ $rc -eq 0 ] || exit $rc
      done <<SETS
${PMC_SETS:-FETCH_SIZE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES
WRITE_SIZE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_INSTS_MFMA}
SETS
      python3 scripts/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_summary.txt 2>&1
      rc=$?; head -30 gpurun_out/pmc_summary.txt
      rm -rf gpurun_out/pmc ;;      # raw traces exceed what gpurun copies back
    profq)
      # per-query kernel summaries (tables generated in HBM), one rocprofv3 run
      # per query set in QS (space separated, e.g. QS="9 10 13 21")
      for q in ${QS:-9 10 13 21 5 18}; do
        IGLOO_PROF_GAP=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$R/gpurun_out/profq_$q" -o run -- python3 "$R/bench.py" --source hbm --queries $q --steps 3 --warmup 5 \
          --eager-steps 0 --vary-params 0 > gpurun_out/profq_$q.log 2>&1
        rc=$?; echo "profq $q rc=$rc"; [ $rc -eq 0 ] || exit $rc
        T=$(find gpurun_out/profq_$q -name "*kernel_trace.csv" | head -1)
        python3 scripts/kernel_summary.py "$T" --steps 3 --top 25 ${KD:+--dispatches "$KD"} > gpurun_out/profq_${q}_summary.txt
        rm -rf gpurun_out/profq_$q; head -8 gpurun_out/profq_${q}_summary.txt
      done ;;
    profspmd)
      # per-query kernel summaries of the SPMD path on one GPU (bench.py with
      # IGLOO_FORCE_SPMD=1: every collective real), one rocprofv3 run per set
      for q in ${QS:-20 22}; do
        IGLOO_FORCE_SPMD=1 IGLOO_PROF_GAP=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$R/gpurun_out/profspmd_$q" -o run -- python3 "$R/bench.py" --source hbm --queries $q --steps 3 \
          --warmup 5 --eager-steps 0 --vary-params 0 > gpurun_out/profspmd_$q.log 2>&1
        rc=$?; echo "profspmd $q rc=$rc"; [ $rc -eq 0 ] || exit $rc
        T=$(find gpurun_out/profspmd_$q -name "*kernel_trace.csv" | head -1)
        python3 scripts/kernel_summary.py "$T" --steps 3 --top 25 > gpurun_out/profspmd_${q}_summary.txt
        rm -rf gpurun_out/profspmd_$q; head -8 gpurun_out/profspmd_${q}_summary.txt
      done ;;
    jitcache)
      # compile the suite's query-specialised kernels at the benchmark scale
      # into gpurun_out/jit_cache (copied into igloo_amd/_jit_cache/ afterwards)
      IGLOO_JIT_CACHE="$R/gpurun_out/jit_cache" IGLOO_JIT_AOT=/nonexistent timeout -k 10 900 python -u bench.py \
        --steps 1 --warmup 1 --eager-steps 0 --vary-params 0 > gpurun_out/jitcache.log 2>&1
      rc=$?; echo "jitcache rc=$rc"; ls gpurun_out/jit_cache | wc -l ;;
    jitsources)
      # record the source of every query-specialised kernel the suite generates
      # at SF100 (validation parameters + two ad-hoc parameter streams whose
      # seeds differ from the ones bench.py times) into gpurun_out/jit_sources;
      # committed as igloo_amd/jit_sources, compiled ahead of time by build()
      # (igloo_amd/ops/jit.py aot_compile)
      IGLOO_DEBUG="jit_dump=$R/gpurun_out/jit_sources" IGLOO_JIT_AOT=/nonexistent timeout -k 10 900 python -u bench.py \
        --steps 1 --warmup 1 --eager-steps 0 --vary-params 2 --param-seed 7000 > gpurun_out/jitsources.log 2>&1
      rc=$?; echo "jitsources rc=$rc"; ls gpurun_out/jit_sources | wc -l ;;
    jitdiff)
      # generated kernels the timed ad-hoc streams request (to compare with
      # igloo_amd/jit_sources: parameter-dependent kernel sources)
      IGLOO_DEBUG="jit_dump=$R/gpurun_out/jit_b" timeout -k 10 900 python -u bench.py \
        --steps 1 --warmup 1 --eager-steps 0 --vary-params 2 > gpurun_out/jitdiff.log 2>&1
      rc=$?; echo "jitdiff rc=$rc"; ls gpurun_out/jit_b | wc -l ;;
    budget)
      # all 22 queries at SF${SF:-10} with the device capped at 1 GB (morsels, spill, external sort)
      timeout -k 10 900 python -u scripts/budget_check.py --sf ${SF:-10} --cap-gb 1 --budget-gb 0.25 --ref gpu \
        --json gpurun_out/budget_sf${SF:-10}.json > gpurun_out/budget_sf${SF:-10}.log 2>&1
      rc=$?; echo "budget rc=$rc"; tail -3 gpurun_out/budget_sf${SF:-10}.log ;;
    share2)
      # two ranks sharing the one GPU (gloo collectives, host staged) vs one rank, SF1
      timeout -k 10 400 python -u bench.py --sf 1 --steps 10 --warmup 3 --per-query \
        > gpurun_out/bench_sf1_1rank.log 2>&1
      rc=$?; echo "sf1 1-rank rc=$rc"; tail -1 gpurun_out/bench_sf1_1rank.log | cut -c1-200
      [ $rc -eq 0 ] || exit $rc
      IGLOO_BENCH_SHARE_GPU=1 IGLOO_BENCH_DIR=/tmp/igloo_tpch_w2 timeout -k 10 600 python -u -m torch.distributed.run \
        --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --sf 1 \
        --steps 10 --warmup 3 --per-query > gpurun_out/bench_sf1_2rank_shared.log 2>&1
      rc=$?; echo "sf1 2-rank shared rc=$rc"; tail -1 gpurun_out/bench_sf1_2rank_shared.log | cut -c1-200 ;;
    proj)
      # per-query 8-GPU projection from a world-of-one SPMD EXPLAIN ANALYZE at
      # SF100, scaled by the committed SPMD graph-mode per-query times
      timeout -k 10 900 python -u scripts/spmd_projection.py --sf ${SF:-100} \
        --graph-log ${GLOG:-profiles/r4_bench_sf100_spmd_world1_c.log} --json gpurun_out/spmd_projection.json \
        > gpurun_out/spmd_projection.txt 2>&1
      rc=$?; echo "proj rc=$rc"; tail -30 gpurun_out/spmd_projection.txt ;;
    gbench)
      timeout -k 10 300 python -u scripts/gather_bench.py --out gpurun_out/gather_bench.txt \
        > gpurun_out/gather_bench.log 2>&1
      rc=$?; echo "gbench rc=$rc"; tail -20 gpurun_out/gather_bench.txt ;;
    atsites)
      # ATen kernels of the warm suite by igloo call site (torch.profiler)
      timeout -k 10 600 python -u scripts/aten_sites.py --sf ${SF:-100} --top 45 > gpurun_out/aten_sites.txt 2>&1
      rc=$?; echo "atsites rc=$rc"; head -30 gpurun_out/aten_sites.txt ;;
    adhoc)
      # ad-hoc statements (fresh TPC-H parameters): per query wall vs device
      # span per stream, then one stream under cProfile
      timeout -k 10 600 python -u scripts/adhoc_profile.py --sf ${SF:-100} --streams 3 \
        --out gpurun_out/adhoc_profile.txt > gpurun_out/adhoc_profile.log 2>&1
      rc=$?; echo "adhoc rc=$rc"; head -60 gpurun_out/adhoc_profile.txt ;;
    atbytes)
      # ATen ops by engine call site, bytes written (TorchDispatchMode)
      timeout -k 10 600 python -u scripts/aten_bytes.py --sf ${SF:-10} --top 50 > gpurun_out/aten_bytes.txt 2>&1
      rc=$?; echo "atbytes rc=$rc"; head -40 gpurun_out/aten_bytes.txt ;;
    rbsites)
      # blocking readbacks per query and how many are parameter-independent
      timeout -k 10 600 python -u scripts/readback_sites.py --sf ${SF:-10} --streams 2 --stacks \
        --out gpurun_out/readback_sites.txt > gpurun_out/readback_sites.log 2>&1
      rc=$?; echo "rbsites rc=$rc"; head -24 gpurun_out/readback_sites.txt ;;
    gsites)
      timeout -k 10 600 python -u scripts/gather_sites.py --sf ${SF:-100} --queries ${QS:-1-22} --timed \
        --out gpurun_out/gather_sites.txt > gpurun_out/gather_sites.log 2>&1
      rc=$?; echo "gsites rc=$rc"; head -30 gpurun_out/gather_sites.txt ;;
    *) echo "unknown mode $mode"; exit 2 ;;
  esac
  [ $rc -eq 0 ] || exit $rc
done
