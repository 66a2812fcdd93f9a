# round 5 GPU pass k: pack_pad_multiple 1024 / 512 (fewer dummy tokens; the new packed lengths run
# hipBLASLt's default solutions, the 2048-multiples have TunableOp entries) vs 2048, interleaved
set -o pipefail
O=gpurun_out/r05/k
mkdir -p $O
bash tools/gpu_ab.sh pad 2 "" "--pad-multiple 1024" "--pad-multiple 512" > $O/pad_ab.txt 2>&1 || { echo "AB FAILED"; cat $O/pad_ab.txt; exit 1; }
cat $O/pad_ab.txt
