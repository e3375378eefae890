set -u
cd "$GRAFT_REPO_ROOT"; ROOT=$(pwd); mkdir -p gpurun_out; export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof_dwt" -o run -- python3 "$ROOT/scripts/bench_paths.py" --only dwt --steps 3 > "$ROOT/gpurun_out/prof_dwt.log" 2>&1
echo rc=$?
