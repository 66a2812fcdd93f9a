# round 5 GPU pass n: va_gate_up_swiglu (fused gate|up GEMM + SwiGLU for the no-grad pass): parity tests,
# kernel A/B at the bench's micro-batch, then bench A/B --fused-mlp-no-grad 0 / 1 interleaved
set -o pipefail
O=gpurun_out/r05/n
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_model_ops_gpu.py tests/test_abi.py -x -v --timeout 300 --timeout-method thread > $O/pytest_model_ops.log 2>&1 || { tail -60 $O/pytest_model_ops.log; exit 1; }
tail -3 $O/pytest_model_ops.log
timeout -k 10 300 python -u tools/gate_up_swiglu_ab.py > $O/gate_up_swiglu_ab.jsonl 2>&1 || { cat $O/gate_up_swiglu_ab.jsonl; exit 1; }
cat $O/gate_up_swiglu_ab.jsonl
bash tools/gpu_ab.sh mlp 2 "" "--fused-mlp-no-grad 1" > $O/bench_mlp_ab.txt 2>&1 || { echo "AB FAILED"; tail -30 $O/bench_mlp_ab.txt; exit 1; }
cat $O/bench_mlp_ab.txt
