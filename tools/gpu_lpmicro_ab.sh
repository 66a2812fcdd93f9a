#!/bin/bash
# A/B of the no-grad log-prob pass micro-batch (log_prob_micro_batch_size_per_gpu) on the headline bench
set -u
O=gpurun_out/lpmicro
mkdir -p $O
for M in 128 256 512 128; do
  timeout -k 10 400 python bench.py --logprob-micro $M --steps 3 --warmup 1 --no-cpu-baseline --out $O/m$M.json > $O/m$M.log 2>&1 || exit $?
  python3 -c "import json;d=json.load(open('$O/m$M.json'));print($M, d['value'], d['ms_per_step'], d['config']['peak_hbm_gb'])"
done
