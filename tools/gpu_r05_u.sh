# round 5 GPU pass u: bench A/B of the weight-gradient MFMA form (--tune 20=16 vs default 32), interleaved
set -o pipefail
O=gpurun_out/r05/u
mkdir -p $O
bash tools/gpu_ab.sh wgrad_mfma 2 "" "--tune 20=16" > $O/bench_wgrad_mfma_ab.txt 2>&1 || { echo "AB FAILED"; tail -30 $O/bench_wgrad_mfma_ab.txt; exit 1; }
cat $O/bench_wgrad_mfma_ab.txt
