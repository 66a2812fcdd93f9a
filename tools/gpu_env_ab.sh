#!/bin/bash
# HIP runtime environment A/B on the headline bench (interleaved, same box): HIP_FORCE_DEV_KERNARG
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/envab
mkdir -p $O
i=0
for kv in 1 0 1 0; do
  i=$((i+1))
  HIP_FORCE_DEV_KERNARG=$kv timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --out $O/b_$i.json > $O/b_$i.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('$O/b_$i.json'));print('HIP_FORCE_DEV_KERNARG=$kv', d['value'], d['ms_per_step'])"
done
for kv in 1 0; do
  i=$((i+1))
  HIP_FORCE_DEV_KERNARG=$kv timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --prompts 8 --out $O/b_$i.json > $O/b_$i.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('$O/b_$i.json'));print('prompts=8 HIP_FORCE_DEV_KERNARG=$kv', d['value'], d['ms_per_step'])"
done
