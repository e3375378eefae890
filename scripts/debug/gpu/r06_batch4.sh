#!/bin/bash
# Round 6 batch 4: deflate occupancy variants (2 strips per workgroup, smaller windows, VGPR cap) ABBA.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u scripts/debug/zvar_ab.py 256 6 cur lw256 wg2n wg2s > gpurun_out/r06_zab_v5.json 2> gpurun_out/r06_zab_v5.err
rc=$?; echo "zab rc=$rc"; cat gpurun_out/r06_zab_v5.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zab_v5.err; exit $rc; }
