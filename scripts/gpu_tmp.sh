set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u scripts/bench_paths.py --only dwt,dct_decode,dct_encode_pcie,ipp > gpurun_out/paths.jsonl 2> gpurun_out/paths.err
rc=$?; echo "paths rc=$rc"; cat gpurun_out/paths.jsonl | cut -c1-400
