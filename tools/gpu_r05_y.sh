# round 5 GPU pass y: after the sweep's staging rework (step counters, fixed per-lane offsets,
# scalar wave index): f1 vs the step-counter build, the fused gate|up + SwiGLU vs hipBLASLt + the
# streaming SwiGLU, and the bench with / without --fused-mlp-no-grad, interleaved; then parity tests
set -o pipefail
O=gpurun_out/r05/y
mkdir -p $O
OLD=verl_amd/lib/ab/libverl_amd_counters.so
for i in 1 2; do
  VERL_AMD_LIB=$OLD timeout -k 10 120 python tools/f1_ab.py --tag counters >> $O/f1_ab.jsonl 2>> $O/f1_ab.err || { echo "old FAILED"; tail -20 $O/f1_ab.err; exit 1; }
  timeout -k 10 120 python tools/f1_ab.py --tag offsets_sgpr_wave >> $O/f1_ab.jsonl 2>> $O/f1_ab.err || { echo "new FAILED"; tail -20 $O/f1_ab.err; exit 1; }
done
cat $O/f1_ab.jsonl
timeout -k 10 300 python tools/gate_up_swiglu_ab.py --splits auto,7,19 > $O/gate_up_swiglu_ab.jsonl 2> $O/gate_up.err || { echo "gate_up FAILED"; tail -20 $O/gate_up.err; exit 1; }
cat $O/gate_up_swiglu_ab.jsonl
run() { local tag=$1; shift; timeout -k 10 400 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --out $O/bench_$tag.json "$@" > $O/bench_$tag.log 2>&1 || { echo "$tag FAILED"; tail -20 $O/bench_$tag.log; exit 1; }; python -c "import json;d=json.load(open('$O/bench_$tag.json'));print('$tag', d['value'], d['ms_per_step'], d['roofline']['frac'])"; }
run default_1
run fused_mlp_1 --fused-mlp-no-grad
run default_2
run fused_mlp_2 --fused-mlp-no-grad
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_linear_logprob_gpu.py tests/test_model_ops_gpu.py tests/test_reference_protocol_gpu.py tests/test_fused_backends_gpu.py > $O/pytest_f1.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/pytest_f1.log; exit 1; }
tail -3 $O/pytest_f1.log
