# round 5 GPU pass ag: flash forward row sums on the matrix core (a ones A-operand against the P^T
# fragments: lacc = sum of the bf16 P the numerator uses) vs the VALU fp32 row sums (HEAD build),
# interleaved on the bench-shaped micro-batch; then the attention tests
set -o pipefail
O=gpurun_out/r05/ag
mkdir -p $O
for i in 1 2 3; do
  VERL_AMD_LIB=verl_amd/lib/ab/libverl_amd_head.so timeout -k 10 120 python tools/attn_ab.py --tag valu_rowsum >> $O/attn_rowsum_ab.jsonl 2>> $O/attn.err || { echo "old FAILED"; tail -20 $O/attn.err; exit 1; }
  timeout -k 10 120 python tools/attn_ab.py --tag mfma_rowsum >> $O/attn_rowsum_ab.jsonl 2>> $O/attn.err || { echo "new FAILED"; tail -20 $O/attn.err; exit 1; }
done
cat $O/attn_rowsum_ab.jsonl
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py tests/test_actor_gpu.py > $O/pytest_attn.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/pytest_attn.log; exit 1; }
tail -1 $O/pytest_attn.log
