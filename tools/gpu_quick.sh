#!/bin/bash
# GPU box: model-side parity tests (fused ops, attention, fused lm_head), microbench, headline bench.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_model_ops_gpu.py tests/test_attention_gpu.py tests/test_linear_logprob_gpu.py tests/test_actor_gpu.py -x -q > gpurun_out/t_quick.log 2>&1
rc=$?; echo "[tests] rc=$rc"; grep -n "Error\|assert \|passed\|failed" gpurun_out/t_quick.log | head -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/model_microbench.py gfx950 2>&1 | grep -v amdgpu.ids
timeout -k 10 400 python bench.py --no-cpu-baseline --steps 2 --warmup 1 --out gpurun_out/bench_q.json > gpurun_out/bench_q.log 2>&1
echo "[bench] rc=$?"; tail -1 gpurun_out/bench_q.log | cut -c1-300
