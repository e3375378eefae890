#!/bin/bash
# Round 6 batch 14: kernel times of the radix-sort K1 variant (rocprofv3 kernel trace).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06_k1sort_prof -o k -- python3 scripts/debug/zvar_once.py dflt 256 3 > gpurun_out/r06_k1sort_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r06_k1sort_prof.log; exit $rc; }
find gpurun_out/r06_k1sort_prof -name '*kernel_stats.csv' -exec cut -c1-60,200-400 {} \;
