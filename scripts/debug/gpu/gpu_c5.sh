set -u -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ipp_gpu.py tests/test_dist_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/c5_t.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/c5_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --c4-frames 0 > gpurun_out/b_c5.json 2> gpurun_out/b_c5.err; rc=$?
python3 -c "
import json; d=json.loads(open('gpurun_out/b_c5.json').read()); c=d.get('c5_e2e_with_gather'); print(json.dumps(c)[:900])"
exit $rc
