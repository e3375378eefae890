#!/bin/bash
# Selected GPU tests (args = pytest targets), one process, bounded.
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 ${T:-600} python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread "$@" > "$OUT/pytest_sel.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" "$OUT/pytest_sel.log" | tail -40; exit $rc
