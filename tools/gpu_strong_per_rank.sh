#!/bin/bash
# per-rank workload of the strong-scaling bench at N = 2 / 4 / 8 (64 / N prompts x 8 responses),
# run on one GPU as world 1: the throughput each rank can reach before any collective
set -u
O=gpurun_out/strong
mkdir -p $O
for P in 32 16 8; do
  timeout -k 10 300 python bench.py --prompts $P --steps 3 --warmup 1 --no-cpu-baseline --out $O/p$P.json > $O/p$P.log 2>&1 || exit $?
  python3 -c "import json;d=json.load(open('$O/p$P.json'));print($P, d['value'], d['ms_per_step'], d['config'].get('micro_batch', d['config']))"
done
