# round 5 GPU pass at: kernel times of the fused q|k|v + bias + RoPE (bench --fused-qkv 1 under
# rocprofv3 --kernel-trace --stats) next to the unfused q|k|v GEMM + rope_qkv_fwd of the default run
set -o pipefail
O=gpurun_out/r05/at
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o qkv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --fused-qkv 1 --out $O/bench_qkv.json > $O/prof.log 2>&1 || { echo "rocprof FAILED"; tail -30 $O/prof.log; exit 1; }
st=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python tools/prof_summary.py $st > $O/kernel_stats_qkv_summary.txt
grep -i "qkv_rope\|rope_qkv\|MT192\|Bias" $O/kernel_stats_qkv_summary.txt | head -8
find $O -name "*kernel_trace.csv" -delete
