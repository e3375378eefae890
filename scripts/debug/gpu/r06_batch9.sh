#!/bin/bash
# Round 6 batch 9: K1 scatter variants and the side-kernel-free upper bound, ABBA on C4.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u scripts/debug/zvar_ab.py 256 8 dflt k1old k1mix noside > gpurun_out/r06_zab_k1.json 2> gpurun_out/r06_zab_k1.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r06_zab_k1.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zab_k1.err; exit $rc; }
