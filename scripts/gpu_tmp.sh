set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u scripts/ab_dwt.py 0,12 > gpurun_out/ab_dwt_pri_b44.log 2>&1
rc=$?; echo "ab rc=$rc"; tail -3 gpurun_out/ab_dwt_pri_b44.log; [ $rc -eq 0 ] || exit $rc
WAVELET=db5 timeout -k 10 300 python -u scripts/ab_dwt.py 0,12 > gpurun_out/ab_dwt_pri_db5.log 2>&1
rc=$?; echo "ab rc=$rc"; tail -3 gpurun_out/ab_dwt_pri_db5.log
