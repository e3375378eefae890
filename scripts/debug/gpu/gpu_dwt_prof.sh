#!/bin/bash
# C3 (4K, l=5, bior4.4) DWT: bench line, rocprofv3 kernel stats, PMC passes.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python scripts/bench_paths.py --only dwt > gpurun_out/dwt_paths.jsonl 2> gpurun_out/dwt_paths.err
rc=$?; echo "paths rc=$rc"; cat gpurun_out/dwt_paths.jsonl; [ $rc -eq 0 ] || exit $rc
bash scripts/prof_dwt.sh || exit 1
bash scripts/pmc_dwt.sh > gpurun_out/pmc_dwt_summary.txt 2>&1; rc=$?; tail -20 gpurun_out/pmc_dwt_summary.txt; exit $rc
