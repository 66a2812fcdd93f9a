#!/bin/bash
# GPU box: fused model-op parity, actor tests, headline bench with and without fused ops.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_model_ops_gpu.py tests/test_actor_gpu.py -x -q > gpurun_out/t_modelops.log 2>&1
echo "[tests] rc=$?"
tail -3 gpurun_out/t_modelops.log
timeout -k 10 400 python bench.py --no-cpu-baseline --steps 2 --warmup 1 --out gpurun_out/bench_fused.json > gpurun_out/bench_fused.log 2>&1
echo "[bench] rc=$?"
tail -2 gpurun_out/bench_fused.log
