#!/bin/bash
# Round 6 final: the whole -m gpu suite, smoke() and bench.py (as the driver runs them), then the
# headline's rocprofv3 kernel stats and timed-launch summary.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r06f}
bash scripts/debug/gpu/r06_full.sh || exit $?
bash scripts/gpu_headline_prof.sh $TAG
