#!/bin/bash
# Round 6 batch 31: K1's pass-1 output as u16 positions (pass 2 re-hashes) vs u32 keys, ABBA on C4
# with a second load of each library.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python3 -u scripts/debug/zvar_ab.py 256 6 t16 t32 t16b t32b > gpurun_out/r06_zab_tmp16.json 2> gpurun_out/r06_zab_tmp16.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r06_zab_tmp16.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zab_tmp16.err; exit $rc; }
