set -u
cd $GRAFT_REPO_ROOT
ROUNDS=16 timeout -k 10 300 python -u scripts/bench_variants.py 17,0 > gpurun_out/ab_enc.log 2>&1
rc=$?; echo "ab rc=$rc"; tail -3 gpurun_out/ab_enc.log
