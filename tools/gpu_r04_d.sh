# round 4 GPU pass d: kernel trace of the bench step, GEMMs split by grid (which hipBLASLt kernel
# runs the lm_head forward / dgrad / wgrad in the step, and their in-step durations)
set -o pipefail
O=gpurun_out/r04
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace -d $O/prof_step -o step -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --out $O/bench_d_under_rocprof.json > $O/bench_d_prof.log 2>&1 || { echo "rocprof bench FAILED"; tail -30 $O/bench_d_prof.log; exit 1; }
db=$(find $O/prof_step -name "*.db" | head -1)
python tools/rocpd_stats.py $db --by-grid --match Cijk > $O/step_gemms_by_grid.txt
python tools/rocpd_stats.py $db > $O/step_kernels.txt
head -30 $O/step_gemms_by_grid.txt
rm -f $db
