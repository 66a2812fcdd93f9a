# round 4 GPU pass v: dK / dV with inline-asm transposed reads (VA_DKDV_ASM_TR build in
# verl_amd/lib/ab/: the next tile's LDS-DMA stays in flight for the whole query tile) vs the product
# build, interleaved; then the attention GPU tests on the variant build
set -o pipefail
O=gpurun_out/r04/attn_asmtr
mkdir -p $O
V=verl_amd/lib/ab/libverl_amd_asmtr.so
for r in 1 2 3; do
  timeout -k 10 120 python tools/attn_ab.py --tag base >> $O/time.jsonl 2>>$O/err.log || { echo "attn_ab FAILED"; tail $O/err.log; exit 1; }
  VERL_AMD_LIB=$V timeout -k 10 120 python tools/attn_ab.py --tag asmtr >> $O/time.jsonl 2>>$O/err.log || { echo "attn_ab asmtr FAILED"; tail $O/err.log; exit 1; }
done
cat $O/time.jsonl
VERL_AMD_LIB=$V timeout -k 10 500 python -u -m pytest tests/test_attention_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; exit $rc
