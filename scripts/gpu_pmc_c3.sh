#!/bin/bash
# PMC summaries of the C3 DWT encode and decode, bit-exact product and the lifting
# form (scripts/pmc_dwt.sh per case) -> gpurun_out/pmc_c3_{enc,dec}{,_lift}/summary.txt
set -u
cd "$GRAFT_REPO_ROOT"
for L in 0 1; do
  for D in 0 1; do
    LIFT=$L DECODE=$D VARIANT=0 bash scripts/pmc_dwt.sh > /dev/null || exit 1
    S=""; [ $D = 1 ] && S=_dec
    N=gpurun_out/pmc_c3_$([ $D = 1 ] && echo dec || echo enc)$([ $L = 1 ] && echo _lift)
    rm -rf $N; mv gpurun_out/pmc_dwt_v0$S $N; echo "done $N"
  done
done
