set -u
cd $GRAFT_REPO_ROOT
DECODE=1 timeout -k 10 300 python -u scripts/ab_dwt.py 6,0,7,8 > gpurun_out/ab_dwt_dec.log 2>&1
rc=$?; echo "ab rc=$rc"; tail -3 gpurun_out/ab_dwt_dec.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_dwt_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_dwt.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_dwt.log
