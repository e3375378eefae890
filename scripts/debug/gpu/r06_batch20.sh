#!/bin/bash
# Round 6 batch 20: longest-first dispatch of the lazy parse (zlib_lpt_kernel), ABBA on C4.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 -u scripts/debug/zvar_ab.py 256 8 dflt nolpt > gpurun_out/r06_zab_lpt.json 2> gpurun_out/r06_zab_lpt.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r06_zab_lpt.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zab_lpt.err; exit $rc; }
