#!/bin/bash
# A GPU check of the current tree: the named test files (or the whole -m gpu
# suite), then bench.py with its defaults.  Usage: scripts/gpu_check.sh TAG [test files...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; TAG=${1:-chk}; shift || true
mkdir -p $OUT
export TMPDIR=/tmp
T=${*:-tests}
timeout -k 10 900 python -u -m pytest $T -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench_$TAG.json; tail -3 $OUT/bench_$TAG.err; exit $rc
