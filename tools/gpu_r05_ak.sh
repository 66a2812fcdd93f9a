# round 5 GPU pass ak (= v at the closing head): bench variants at HEAD (regression check of the round's changes): realistic
# response lengths, the fused-kernel update pass, the 8-prompt per-rank workload, the sharded optimizer
set -o pipefail
O=gpurun_out/r05/ak
mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 400 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --out $O/bench_$tag.json "$@" > $O/bench_$tag.log 2>&1 || { echo "$tag FAILED"; tail -20 $O/bench_$tag.log; exit 1; }; python -c "import json;d=json.load(open('$O/bench_$tag.json'));print('$tag', d['value'], d['ms_per_step'], d['config']['peak_hbm_gb'], d['final_metrics'].get('actor/pg_clipfrac'))"; }
run realistic --responses realistic
run fused_kernels --fused-kernels 1
run p8 --prompts 8
run zero --zero 1
