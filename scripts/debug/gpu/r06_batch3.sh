#!/bin/bash
# Round 6 batch 3: deflate final form vs p1 (the same switches before the G4DW/FARWAVE code left) vs the product.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u scripts/debug/zvar_ab.py 256 6 p1 final > gpurun_out/r06_zab_v4.json 2> gpurun_out/r06_zab_v4.err
rc=$?; echo "zab rc=$rc"; cat gpurun_out/r06_zab_v4.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zab_v4.err; exit $rc; }
