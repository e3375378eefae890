#!/bin/bash
# rocprofv3 kernel trace + stats of the C3 encode (ab_dwt.py with variant 0 alone), for the timeline.
set -u
cd "$GRAFT_REPO_ROOT"; ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_dwt_trace" -o run -- python3 "$ROOT/scripts/ab_dwt.py" ${ENC:-0} > "$ROOT/gpurun_out/prof_dwt_trace.log" 2>&1
rc=$?; echo rc=$rc; tail -3 "$ROOT/gpurun_out/prof_dwt_trace.log"; exit $rc
