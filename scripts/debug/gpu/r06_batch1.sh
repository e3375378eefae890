#!/bin/bash
# Round 6 batch: deflate variants ABBA, encode SDWA ABBA, DCT decode counters (dense / smooth).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u scripts/debug/zvar_ab.py 256 6 late0 lg lf lgf lgf7168 > gpurun_out/r06_zab_v2.json 2> gpurun_out/r06_zab_v2.err
rc=$?; echo "zab rc=$rc"; cat gpurun_out/r06_zab_v2.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zab_v2.err; exit $rc; }
timeout -k 10 300 python3 -u scripts/lib_ab_encode.py 16 sdwac > gpurun_out/r06_sdwa_ab.json 2> gpurun_out/r06_sdwa_ab.err
rc=$?; echo "sdwa rc=$rc"; cat gpurun_out/r06_sdwa_ab.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_sdwa_ab.err; exit $rc; }
DENSE=1 bash scripts/pmc_r06.sh dct_dec_dense python3 scripts/dct_dec_once.py 2 || exit $?
bash scripts/pmc_r06.sh dct_dec_smooth python3 scripts/dct_dec_once.py 2 || exit $?
echo batch done
