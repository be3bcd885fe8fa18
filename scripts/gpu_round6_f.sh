cd /root/repo && export TMPDIR=/tmp
DBG_SET="igloo_amd.exec.joins.UNIQUE_PAIRS_SORTED=0" timeout -k 10 120 python -u scripts/dbg_spmd_query.py 9 4 0 '[["keyuniq_called_path_off",{},[]]]' > gpurun_out/r6_dbg_q9_side.log 2>&1 || exit 3
bash scripts/mfma_hash_ab.sh > gpurun_out/r6_mfma_ab.log 2>&1
