set -u
cd $GRAFT_REPO_ROOT
AB=0 bash scripts/prof_ab_dwt.sh > /dev/null && echo prof ok && VARIANT=0 bash scripts/pmc_strip.sh > gpurun_out/pmc0.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -8 gpurun_out/pmc0.log | cut -c1-200
