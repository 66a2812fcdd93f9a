# round 5 GPU pass ai: the training forward's gate|up GEMM + SwiGLU as one kernel that also writes the
# projection for the backward (va_gate_up_swiglu_save, ABI 8; actor option fused_mlp_train) — parity
# tests, then the bench with / without --fused-mlp-train 1, interleaved
set -o pipefail
O=gpurun_out/r05/ai
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_model_ops_gpu.py tests/test_linear_logprob_gpu.py > $O/pytest_mlp.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/pytest_mlp.log; exit 1; }
tail -1 $O/pytest_mlp.log
run() { local tag=$1; shift; timeout -k 10 400 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --out $O/bench_$tag.json "$@" > $O/bench_$tag.log 2>&1 || { echo "$tag FAILED"; tail -20 $O/bench_$tag.log; exit 1; }; python -c "import json;d=json.load(open('$O/bench_$tag.json'));r=d['roofline'];print('$tag', d['value'], d['ms_per_step'], d['config']['peak_hbm_gb'], d['final_metrics'].get('actor/pg_loss'), d['final_metrics'].get('actor/grad_norm'))"; }
run default_1
run mlp_train_1 --fused-mlp-train 1
run default_2
run mlp_train_2 --fused-mlp-train 1
