# round 5 GPU pass t: the weight-gradient kernel's 16x16x32 MFMA form (VA_TUNE_WGRAD_MFMA = 16):
# parity tests, then the per-shape A/B against the 32x32x16 form at the bench's token count
set -o pipefail
O=gpurun_out/r05/t
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_weight_grad_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest_wgrad.log 2>&1 || { tail -40 $O/pytest_wgrad.log; exit 1; }
tail -2 $O/pytest_wgrad.log
timeout -k 10 300 python -u tools/wgrad_mfma_ab.py > $O/wgrad_mfma_ab.jsonl 2>&1 || { cat $O/wgrad_mfma_ab.jsonl; exit 1; }
cat $O/wgrad_mfma_ab.jsonl
