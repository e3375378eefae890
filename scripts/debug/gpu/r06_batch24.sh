#!/bin/bash
# Round 6 batch 24: is the load-to-load spread the side stream's early-exit kernels? Library
# copies with and without the side kernels (VCF_ZX_NOSIDE: C4 has no non-lazy strip).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u scripts/debug/zvar_ab.py 256 6 pcopy pcopy2 noside ncopy dflt dcopy > gpurun_out/r06_zab_noside.json 2> gpurun_out/r06_zab_noside.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r06_zab_noside.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zab_noside.err; exit $rc; }
