#!/bin/bash
# caching-allocator expandable segments A/B on the headline bench (interleaved, same box)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/allocab
mkdir -p $O
i=0
for p in 64 64 8; do
  for es in 1 0; do
    i=$((i+1))
    if [ $es = 1 ]; then export PYTORCH_ALLOC_CONF=expandable_segments:True; else unset PYTORCH_ALLOC_CONF; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --prompts $p --out $O/b_$i.json > $O/b_$i.log 2>&1 || exit $?
    python -c "import json;d=json.load(open('$O/b_$i.json'));print('prompts=$p expandable=$es', d['value'], d['ms_per_step'], d['config']['peak_hbm_gb'])"
  done
done
