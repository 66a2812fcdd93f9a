# round 5 GPU pass al: the fused gate|up + SwiGLU storing through a wave-private LDS scratch (whole
# 128-B row segments per store) vs direct 8-byte stores (HEAD build): parity tests, kernel timing,
# and the bench with the no-grad fusion (default) and with the training fusion too, interleaved
set -o pipefail
O=gpurun_out/r05/al
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_model_ops_gpu.py > $O/pytest_mlp.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/pytest_mlp.log; exit 1; }
tail -1 $O/pytest_mlp.log
for v in base new; do
  if [ $v = base ]; then export VERL_AMD_LIB=verl_amd/lib/ab/libverl_amd_base.so; else unset VERL_AMD_LIB; fi
  timeout -k 10 300 python tools/gate_up_swiglu_ab.py --splits auto > $O/gate_up_$v.jsonl 2> $O/gate_up_$v.err || { echo "gate_up $v FAILED"; tail -20 $O/gate_up_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$O/gate_up_$v.jsonl'));print('$v', d['median_ms'])"
done
unset VERL_AMD_LIB
run() { local tag=$1; shift; timeout -k 10 400 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --out $O/bench_$tag.json "$@" > $O/bench_$tag.log 2>&1 || { echo "$tag FAILED"; tail -20 $O/bench_$tag.log; exit 1; }; python -c "import json;d=json.load(open('$O/bench_$tag.json'));print('$tag', d['value'], d['ms_per_step'])"; }
base() { VERL_AMD_LIB=verl_amd/lib/ab/libverl_amd_base.so VERL_AMD_LIB_AB=1 run "$@"; }
base base_default_1
run new_default_1
run new_mlp_train_1 --fused-mlp-train 1
base base_default_2
run new_default_2
run new_mlp_train_2 --fused-mlp-train 1
