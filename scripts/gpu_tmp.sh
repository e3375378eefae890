set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u scripts/ab_dwt.py 0,1,6 > gpurun_out/ab_dwt.log 2>&1
rc=$?; echo "ab rc=$rc"; tail -3 gpurun_out/ab_dwt.log; [ $rc -eq 0 ] || exit $rc
true

