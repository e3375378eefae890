set -e
cd $GRAFT_REPO_ROOT
for F in 64 60 61 64 128 60 64; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --frames $F --steps 200 > gpurun_out/tail_$F.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/tail_$F.json'));print($F, d['ms_per_step'], d['value'], d['roofline']['kernel_ms_per_launch']/$F*64)"
done
