# round 4 GPU pass q: the per-rank workloads of the driver's strong-scaling runs, at N = 1 on one GPU
# (N = 2 / 4 / 8 give each rank 32 / 16 / 8 prompts x 8 responses): the compute side of the scaling
# curve without the gradient all-reduce
set -o pipefail
O=gpurun_out/r04/scale_proxy
mkdir -p $O
for p in 32 16 8; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --prompts $p --no-cpu-baseline --out $O/prompts$p.json > $O/prompts$p.log 2>&1 || { echo "bench prompts $p FAILED"; tail -20 $O/prompts$p.log; exit 1; }
  python -c "import json;d=json.load(open('$O/prompts$p.json'));print($p, d['value'], d['ms_per_step'], d['config'].get('compute_micro_batch'))"
done
