#!/bin/bash
# The whole -m gpu suite (one process) and __graft_entry__.smoke(), as the driver runs them.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; TAG=${1:-suite}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke_$TAG.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke_$TAG.log; exit $rc
