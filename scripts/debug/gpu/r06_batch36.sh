#!/bin/bash
# Round 6 batch 36: the 9 216-byte window's shift slack (1024 / 512 / 256 bytes), ABBA on C4, and the
# parse's phase clocks with the window laid over the flush-only LDS.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python3 -u scripts/debug/zvar_ab.py 256 6 base sl512 sl256 > gpurun_out/r06_zab_slack.json 2> gpurun_out/r06_zab_slack.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/r06_zab_slack.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zab_slack.err; exit $rc; }
timeout -k 10 240 python3 -u scripts/debug/zprof_run.py 256 > gpurun_out/r06_zprof_alias.json 2> gpurun_out/r06_zprof_alias.err
rc=$?; echo "zprof rc=$rc"; cat gpurun_out/r06_zprof_alias.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/r06_zprof_alias.err; exit $rc; }
