# round 5 GPU pass ar: the q|k|v GEMM + bias + RoPE as one kernel (va_qkv_rope, ABI 9; option
# fused_qkv): parity tests, then the bench with / without --fused-qkv 1, interleaved
set -o pipefail
O=gpurun_out/r05/ar
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_model_ops_gpu.py -k "qkv or rope" > $O/pytest_qkv.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/pytest_qkv.log; exit 1; }
tail -1 $O/pytest_qkv.log
run() { local tag=$1; shift; timeout -k 10 400 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --out $O/bench_$tag.json "$@" > $O/bench_$tag.log 2>&1 || { echo "$tag FAILED"; tail -20 $O/bench_$tag.log; exit 1; }; python -c "import json;d=json.load(open('$O/bench_$tag.json'));print('$tag', d['value'], d['ms_per_step'], d['final_metrics'].get('actor/grad_norm'))"; }
run default_1
run qkv_1 --fused-qkv 1
run default_2
run qkv_2 --fused-qkv 1
