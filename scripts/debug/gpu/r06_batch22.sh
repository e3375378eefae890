#!/bin/bash
# Round 6 batch 22: K1 pass-1 counts four positions per lane, ABBA on C4.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u scripts/debug/zvar_ab.py 256 8 dflt quad > gpurun_out/r06_zab_quad.json 2> gpurun_out/r06_zab_quad.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r06_zab_quad.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zab_quad.err; exit $rc; }
