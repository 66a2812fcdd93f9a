# round 4 GPU pass c: interleaved A/B of the weight-gradient remainder tiles (VA_TUNE_WGRAD_REMAINDER
# = 18), the bench with use_fused_kernels (fused lm_head backward: time and peak HBM), and the
# lm_head forward GEMM gap probe (plain vs TunableOp table) with a rocprofv3 kernel trace
set -o pipefail
O=gpurun_out/r04
mkdir -p $O
for arm in rem1 rem0 rem1 rem0; do
  t=""; [ $arm = rem0 ] && t="--tune 18=0"
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline $t --out $O/bench_c_$arm.json > $O/bench_c_$arm.log 2>&1 || { echo "bench $arm FAILED"; tail -30 $O/bench_c_$arm.log; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_c_$arm.json'));print('$arm', d['value'], d['ms_per_step'])" | tee -a $O/bench_wgrad_remainder_ab.txt
done
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --fused-kernels 1 --out $O/bench_c_fused.json > $O/bench_c_fused.log 2>&1 || { echo "bench fused FAILED"; tail -30 $O/bench_c_fused.log; exit 1; }
python -c "import json;d=json.load(open('$O/bench_c_fused.json'));print('fused', d['value'], d['ms_per_step'], d['config']['peak_hbm_gb'])"
timeout -k 10 300 python tools/lm_head_gap.py > $O/lm_head_gap.json 2>$O/lm_head_gap.err || { echo "lm_head_gap FAILED"; tail -20 $O/lm_head_gap.err; exit 1; }
cat $O/lm_head_gap.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_lm_head_gap -o lm_head_gap -- python tools/lm_head_gap.py > $O/lm_head_gap_prof.log 2>&1 || { echo "rocprof lm_head_gap FAILED"; tail -20 $O/lm_head_gap_prof.log; exit 1; }
find $O/prof_lm_head_gap -name "*kernel_stats.csv"
