#!/bin/bash
# instruction-cache counters per encode variant: scripts/pmc_ic.sh "1 7"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_ic; mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
for v in ${1:-1}; do
  for grp in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ" "SQ_IFETCH SQ_IFETCH_LEVEL SQC_ICACHE_BUSY_CYCLES"; do
    tag=$(echo $grp | cut -c1-12 | tr ' ' '_')
    timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/v${v}_$tag" -o pmc \
        -- python3 "$ROOT/bench.py" --no-cpu-baseline --steps 3 --warmup 1 --variant $v > "$OUT/v${v}_$tag.log" 2>&1
    rc=$?; echo "v$v [$grp] rc=$rc"; case $rc in 0) ;; 124|134|137|139) exit $rc;; *) tail -3 "$OUT/v${v}_$tag.log";; esac
  done
done
python3 - "$OUT" << 'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
for v in sorted({os.path.basename(d).split('_')[0] for d in glob.glob(out + '/v*_*') if os.path.isdir(d)}):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{out}/{v}_*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(v, {k: round(sum(x) / len(x)) for k, x in sorted(acc.items())})
PY
