# round 5 GPU pass f: flash forward without the max exchange when no lane needs a rescale and with
# per-lane row-sum halves; dK/dV with -delta staged (no per-element negation): attention parity,
# attn_ab against the previous library, interleaved; the fused lm_head default mode against torch
set -o pipefail
O=gpurun_out/r05/f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_attention_gpu.py tests/test_reference_protocol_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest FAILED"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  VERL_AMD_LIB=verl_amd/lib/ab/lib_base.so timeout -k 10 200 python tools/attn_ab.py --tag base >> $O/attn_ab.jsonl 2>> $O/attn_ab.err || { echo "attn base FAILED"; tail $O/attn_ab.err; exit 1; }
  timeout -k 10 200 python tools/attn_ab.py --tag new >> $O/attn_ab.jsonl 2>> $O/attn_ab.err || { echo "attn new FAILED"; tail $O/attn_ab.err; exit 1; }
done
cut -c1-220 $O/attn_ab.jsonl
