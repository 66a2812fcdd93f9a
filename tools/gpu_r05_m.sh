# round 5 GPU pass m: the probe of pass l plus one wave per SIMD (4 waves of 128 x 128 tiles,
# accumulators in registers via -amdgpu-mfma-vgpr-form=1, spilling into AGPRs)
set -o pipefail
O=gpurun_out/r05/m
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kats_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest_kats.log 2>&1 || { tail -40 $O/pytest_kats.log; exit 1; }
tail -3 $O/pytest_kats.log
B=tools/bin/t256_mfma_ab
timeout -k 10 150 $B 131072 896 151936 8 5 > $O/mfma_lm_head.jsonl 2>&1 || { cat $O/mfma_lm_head.jsonl; exit 1; }
cat $O/mfma_lm_head.jsonl
for s in 2 19; do
  timeout -k 10 60 $B 151552 896 9728 $s 7 >> $O/mfma_gate_up.jsonl 2>&1 || { cat $O/mfma_gate_up.jsonl; exit 1; }
done
cat $O/mfma_gate_up.jsonl
