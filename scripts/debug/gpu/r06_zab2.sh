#!/bin/bash
# Round 6: ABBA of deflate variants against the product on the C4 workload.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u scripts/debug/zvar_ab.py 256 6 $ZVARS > gpurun_out/r06_zab_$TAG.json 2> gpurun_out/r06_zab_$TAG.err
rc=$?; echo "zab rc=$rc"; cat gpurun_out/r06_zab_$TAG.json; tail -3 gpurun_out/r06_zab_$TAG.err; exit $rc
