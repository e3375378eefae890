set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
VCF_ZLIB_SLOTS=1 timeout -k 10 200 python -u scripts/zprof_run.py 64 > gpurun_out/zp64.json || exit $?
cat gpurun_out/zp64.json
VCF_ZLIB_SLOTS=1 timeout -k 10 200 python -u scripts/zprof_run.py 256 > gpurun_out/zp256.json || exit $?
cat gpurun_out/zp256.json
VCF_ZLIB_SLOTS=3 timeout -k 10 300 python -u scripts/zdbg.py 256 gpurun_out/zd3.npz || exit $?
VCF_ZLIB_SLOTS=3 timeout -k 10 300 python -u scripts/zdbg.py 256 gpurun_out/zd3b.npz || exit $?
