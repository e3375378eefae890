set -u -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for L in libvcf_zprof.so libvcf_zprof_pad3.so libvcf_zprof_pad2.so; do
  ZPROF_LIB=$L timeout -k 10 200 python -u scripts/zprof_run.py 256 || exit $?
done
