set -u
cd "$GRAFT_REPO_ROOT"; ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp; cd /tmp
rm -rf /tmp/prof_dwt; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_dwt -o run -- python3 "$ROOT/scripts/bench_paths.py" --only dwt --dwt-variants 0 --steps 3 > "$ROOT/gpurun_out/prof_dwt.log" 2>&1
rc=$?; echo rc=$rc; mkdir -p "$ROOT/gpurun_out/prof_dwt"; cp $(find /tmp/prof_dwt -name "*kernel_stats.csv") "$ROOT/gpurun_out/prof_dwt/" ; exit $rc
