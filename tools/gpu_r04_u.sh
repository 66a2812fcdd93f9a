# round 4 GPU pass u: dK / dV kernel with the row-constant load issued before the LDS-DMA and
# unconditional (hipcc no longer drains the DMA at the top of each query tile): attention timing
# (defaults vs register staging), then the attention GPU tests
set -o pipefail
O=gpurun_out/r04/attn_dkdv
mkdir -p $O
for r in 1 2 3; do
  for d in 7 3; do
    timeout -k 10 120 python tools/attn_ab.py --tag dma$d --tune 19=$d >> $O/time.jsonl 2>>$O/err.log || { echo "attn_ab FAILED"; tail $O/err.log; exit 1; }
  done
done
cat $O/time.jsonl
timeout -k 10 500 python -u -m pytest tests/test_attention_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; exit $rc
