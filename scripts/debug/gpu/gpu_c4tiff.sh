set -u -o pipefail
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_dist_gpu.py::test_bench_c4_block_small -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_z2.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_z2.log | tail -30
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_c4t.json 2> gpurun_out/bench_c4t.err
rc=$?; echo "bench rc=$rc"; tail -c 2500 gpurun_out/bench_c4t.json; tail -3 gpurun_out/bench_c4t.err; exit $rc
