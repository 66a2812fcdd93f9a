#!/bin/bash
# bucket clip vs torch's per-parameter clip: tests, then the N=8 per-rank workload (8 prompts) and the
# N=1 workload, interleaved on one box
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/clip
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_actor_gpu.py tests/test_zero_gpu.py tests/test_critic_gpu.py tests/test_nonfinite_skip.py tests/test_trainer_step_gpu.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
i=0
for p in 8 8 64; do
  for tc in 1 0; do
    i=$((i+1))
    VERL_AMD_TORCH_CLIP=$tc timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --prompts $p \
      --out $O/b_$i.json > $O/b_$i.log 2>&1 || exit $?
    python -c "import json;d=json.load(open('$O/b_$i.json'));print('prompts=$p torch_clip=$tc', d['value'], d['ms_per_step'])"
  done
done
