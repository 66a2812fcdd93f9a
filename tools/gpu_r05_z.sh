# round 5 GPU pass z: the bench with / without --fused-mlp-no-grad 1 after the sweep's staging
# rework, interleaved; then the f1 / model-ops parity tests
set -o pipefail
O=gpurun_out/r05/z
mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 400 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --out $O/bench_$tag.json "$@" > $O/bench_$tag.log 2>&1 || { echo "$tag FAILED"; tail -20 $O/bench_$tag.log; exit 1; }; python -c "import json;d=json.load(open('$O/bench_$tag.json'));print('$tag', d['value'], d['ms_per_step'], d['roofline']['frac'])"; }
run default_1
run fused_mlp_1 --fused-mlp-no-grad 1
run default_2
run fused_mlp_2 --fused-mlp-no-grad 1
run default_3
run fused_mlp_3 --fused-mlp-no-grad 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_linear_logprob_gpu.py tests/test_model_ops_gpu.py tests/test_reference_protocol_gpu.py tests/test_fused_backends_gpu.py > $O/pytest_f1.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/pytest_f1.log; exit 1; }
tail -3 $O/pytest_f1.log
