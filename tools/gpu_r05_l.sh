# round 5 GPU pass l: MFMA-shape probe of the f1 sweep (tools/t256_mfma_ab.hip; prebuilt into
# tools/bin/ on the CPU side): 16x16x32 vs 32x32x16, core-only and with the f1 statistics epilogue,
# at the lm_head shape and the gate|up shape
set -o pipefail
O=gpurun_out/r05/l
mkdir -p $O
B=tools/bin/t256_mfma_ab
timeout -k 10 120 $B 131072 896 151936 8 5 > $O/mfma_lm_head.jsonl 2>&1 || { cat $O/mfma_lm_head.jsonl; exit 1; }
cat $O/mfma_lm_head.jsonl
for s in 1 2 19 38; do
  timeout -k 10 60 $B 151552 896 9728 $s 7 >> $O/mfma_gate_up.jsonl 2>&1 || { cat $O/mfma_gate_up.jsonl; exit 1; }
done
cat $O/mfma_gate_up.jsonl
