# round 5 GPU pass ae: flash attention softmax in packed fp32 (forward: v_pk_fma_f32 / v_pk_add_f32
# for the score FMAs and the two running row sums; dQ backward: packed score FMAs) vs the previous
# build, interleaved on the bench-shaped micro-batch; checksums must match; then the attention tests
set -o pipefail
O=gpurun_out/r05/ae
mkdir -p $O
for i in 1 2 3; do
  VERL_AMD_LIB=verl_amd/lib/ab/libverl_amd_prepk.so timeout -k 10 120 python tools/attn_ab.py --tag scalar >> $O/attn_pk_ab.jsonl 2>> $O/attn.err || { echo "old FAILED"; tail -20 $O/attn.err; exit 1; }
  timeout -k 10 120 python tools/attn_ab.py --tag packed >> $O/attn_pk_ab.jsonl 2>> $O/attn.err || { echo "new FAILED"; tail -20 $O/attn.err; exit 1; }
done
cat $O/attn_pk_ab.jsonl
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py > $O/pytest_attn.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/pytest_attn.log; exit 1; }
tail -1 $O/pytest_attn.log
