# round 5 GPU pass o: SwiGLU kernels on the hardware reciprocal (va_sigmoid / va_silu, no IEEE division):
# model-op parity tests, then the fused gate|up + SwiGLU kernel A/B; the bench A/B only if the fused
# kernel beats the unfused pair
set -o pipefail
O=gpurun_out/r05/o
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_model_ops_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest_model_ops.log 2>&1 || { tail -60 $O/pytest_model_ops.log; exit 1; }
tail -3 $O/pytest_model_ops.log
timeout -k 10 300 python -u tools/gate_up_swiglu_ab.py --splits auto,7,19,38 > $O/gate_up_swiglu_ab.jsonl 2>&1 || { cat $O/gate_up_swiglu_ab.jsonl; exit 1; }
cat $O/gate_up_swiglu_ab.jsonl
python - <<'PY' || exit 0
import json
d = json.loads(open("gpurun_out/r05/o/gate_up_swiglu_ab.jsonl").read().strip().splitlines()[-1])
m = d["median_ms"]
best = min(v for k, v in m.items() if k.startswith("fused"))
print("fused best", best, "unfused", m["unfused_gemm_plus_swiglu"])
raise SystemExit(0 if best < m["unfused_gemm_plus_swiglu"] else 1)
PY
bash tools/gpu_ab.sh mlp 2 "" "--fused-mlp-no-grad 1" > $O/bench_mlp_ab.txt 2>&1 || { echo "AB FAILED"; tail -30 $O/bench_mlp_ab.txt; exit 1; }
cat $O/bench_mlp_ab.txt
