#!/bin/bash
# timed-region sensitivity to the number of untimed warmup steps (full batch and the N = 8 per-rank
# workload), same box
set -u
O=gpurun_out/wuab
mkdir -p $O
for cfg in "64 1 3" "64 2 3" "8 1 3" "8 2 3" "8 1 6"; do
  set -- $cfg
  P=$1; W=$2; K=$3
  timeout -k 10 300 python bench.py --prompts $P --steps $K --warmup $W --no-cpu-baseline \
    --out $O/p${P}_w${W}_k$K.json > $O/p${P}_w${W}_k$K.log 2>&1 || exit $?
  python3 -c "import json;d=json.load(open('$O/p${P}_w${W}_k$K.json'));print('prompts $P warmup $W steps $K', d['value'], d['ms_per_step'])"
  grep "step" $O/p${P}_w${W}_k$K.log | grep -v '^{' | tail -8
done
