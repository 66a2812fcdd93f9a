# round 4 GPU pass x: the f1 forward's vocab ranges per row block in the bench step
# (VERL_AMD_LINEAR_LOGPROB_SPLITS 2 / 4 / 8 = default at 131,072 rows), interleaved: in-step f1
# time (the line's roofline_f1) and step throughput
set -o pipefail
O=gpurun_out/r04/f1_splits_step
mkdir -p $O
for r in 1 2; do
  for sp in 8 4 2; do
    VERL_AMD_LINEAR_LOGPROB_SPLITS=$sp timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --out $O/s${sp}_r$r.json > $O/s${sp}_r$r.log 2>&1 || { echo "bench splits $sp FAILED"; tail -20 $O/s${sp}_r$r.log; exit 1; }
    python -c "import json;d=json.load(open('$O/s${sp}_r$r.json'));f=d['roofline_f1'];print($sp, d['value'], d['ms_per_step'], f['avg_launch_us'], f['frac'])"
  done
done
