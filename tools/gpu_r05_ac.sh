# round 5 GPU pass ac: the f1 sweep with its staging between the K-halves (product build) — parity
# tests of every sweep user, f1 / fused gate|up timings, and the bench with / without the fused MLP
set -o pipefail
O=gpurun_out/r05/ac
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_linear_logprob_gpu.py tests/test_model_ops_gpu.py tests/test_reference_protocol_gpu.py tests/test_fused_backends_gpu.py tests/test_kats_gpu.py > $O/pytest_f1.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/pytest_f1.log; exit 1; }
tail -2 $O/pytest_f1.log
for i in 1 2; do
  VERL_AMD_LIB=verl_amd/lib/ab/libverl_amd_base.so timeout -k 10 120 python tools/f1_ab.py --tag base >> $O/f1_ab.jsonl 2>> $O/f1_ab.err || { echo "base FAILED"; exit 1; }
  timeout -k 10 120 python tools/f1_ab.py --tag product >> $O/f1_ab.jsonl 2>> $O/f1_ab.err || { echo "product FAILED"; tail -20 $O/f1_ab.err; exit 1; }
done
python -c "
import json
for l in open('$O/f1_ab.jsonl'): d=json.loads(l); print(d['tag'], d['ms_median'], d['tflops'])"
timeout -k 10 300 python tools/gate_up_swiglu_ab.py --splits auto,7,19 > $O/gate_up_swiglu_ab.jsonl 2> $O/gate_up.err || { echo "gate_up FAILED"; tail -20 $O/gate_up.err; exit 1; }
python -c "import json;d=json.load(open('$O/gate_up_swiglu_ab.jsonl'));print(d['median_ms'])"
run() { local tag=$1; shift; timeout -k 10 400 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --out $O/bench_$tag.json "$@" > $O/bench_$tag.log 2>&1 || { echo "$tag FAILED"; tail -20 $O/bench_$tag.log; exit 1; }; python -c "import json;d=json.load(open('$O/bench_$tag.json'));r=d['roofline'];print('$tag', d['value'], d['ms_per_step'], r['frac'], r.get('launch_us_min_median_max'))"; }
run default_1
run fused_mlp_1 --fused-mlp-no-grad 1
run default_2
run fused_mlp_2 --fused-mlp-no-grad 1
