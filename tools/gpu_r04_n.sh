# round 4 GPU pass n: flash attention with LDS-DMA staging (VA_TUNE_FLASH_DMA = 19: bit 1 forward
# K / V, bit 2 dQ K / V, bit 4 dK / dV Q / dO) vs register staging, interleaved, with the dQ key
# block (VA_TUNE_FLASH_DQ_KB = 10) and dK / dV query tile (VA_TUNE_FLASH_DKDV_QT = 9) choices that
# change occupancy; the checksums must agree; then the attention GPU tests
set -o pipefail
O=gpurun_out/r04/attn_dma
mkdir -p $O
for r in 1 2; do
  for cfg in "0 128 128" "1 128 128" "3 128 128" "3 64 128" "7 64 128" "7 64 64" "0 128 128"; do
    set -- $cfg
    timeout -k 10 120 python tools/attn_ab.py --tag dma$1_dq$2_qt$3 --tune 19=$1 --tune 10=$2 --tune 9=$3 >> $O/time.jsonl 2>>$O/err.log || { echo "attn_ab $cfg FAILED"; tail $O/err.log; exit 1; }
  done
done
cat $O/time.jsonl
timeout -k 10 500 python -u -m pytest tests/test_attention_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; exit $rc
