#!/bin/bash
# N = 8 per-rank workload (8 prompts x 8 responses, one 64-response micro-batch) on one GPU:
# input-gradient layout A/B (VERL_AMD_DGRAD_LAYOUT), interleaved
set -u
O=gpurun_out/p8ab
mkdir -p $O
i=0
for L in nn tn nn tn; do
  i=$((i + 1))
  VERL_AMD_DGRAD_LAYOUT=$L timeout -k 10 300 python bench.py --prompts 8 --steps 5 --warmup 2 --no-cpu-baseline \
    --out $O/$L$i.json > $O/$L$i.log 2>&1 || exit $?
  python3 -c "import json;d=json.load(open('$O/$L$i.json'));print('$L', d['value'], d['ms_per_step'])"
done
