# round 4, second GPU pass: fused lm_head backward A/B (kernel + whole pass, peak HBM), the -m gpu
# suite, smoke(), then the bench with the default (unfused update pass) and with use_fused_kernels
set -o pipefail
O=gpurun_out/r04
mkdir -p $O
# (f1_bwd_ab measured in the previous call: gpurun_out/r04/f1_bwd_ab_b.json)

export VA_REHEARSAL_OUT=$O/rehearsal
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 700 --timeout-method thread > $O/pytest_gpu_b.log 2>&1 || { echo "pytest FAILED"; tail -60 $O/pytest_gpu_b.log; exit 1; }
tail -3 $O/pytest_gpu_b.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_b.log 2>&1 || { echo "smoke FAILED"; tail -30 $O/smoke_b.log; exit 1; }
tail -2 $O/smoke_b.log
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --out $O/bench_b_default.json > $O/bench_b_default.log 2>&1 || { echo "bench default FAILED"; tail -30 $O/bench_b_default.log; exit 1; }
head -c 700 $O/bench_b_default.json; echo
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --fused-kernels 1 --no-cpu-baseline --out $O/bench_b_fused.json > $O/bench_b_fused.log 2>&1 || { echo "bench fused FAILED"; tail -30 $O/bench_b_fused.log; exit 1; }
head -c 700 $O/bench_b_fused.json; echo
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python tools/lm_head_gap.py > $O/lm_head_gap.json 2>$O/lm_head_gap.err || { echo "lm_head_gap FAILED"; tail -20 $O/lm_head_gap.err; exit 1; }
cat $O/lm_head_gap.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_lm_head_gap -o lm_head_gap -- python tools/lm_head_gap.py > $O/lm_head_gap_prof.log 2>&1 || { echo "rocprof lm_head_gap FAILED"; tail -20 $O/lm_head_gap_prof.log; exit 1; }
find $O/prof_lm_head_gap -name "*kernel_stats.csv" | head -3
