#!/bin/bash
# The lifting DWT path: GPU tests, kernel stats, then bench.py's C3 block alone
# (headline short, C2/C4/C5 off) for the lifting leg next to the bit-exact one.
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/debug/gpu/gpu_lift.sh || exit $?
timeout -k 10 400 python3 bench.py --steps 10 --warmup 5 --c4-frames 0 --c5-frames 0 --c2-reps 0 \
    > gpurun_out/lift_bench.json 2> gpurun_out/lift_bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/lift_bench.err; exit $rc; }
python3 -c "import json; d=json.loads(open('gpurun_out/lift_bench.json').read().strip().splitlines()[-1]); c=d['c3_dwt']; print(json.dumps({k: c.get(k) for k in ('encode','decode','lifting','error','check')}, indent=1)[:3000])"
