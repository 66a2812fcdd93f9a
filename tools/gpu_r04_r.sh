# round 4 GPU pass r: the N = 8 per-rank workload (8 prompts x 8 responses) at N = 1 under a kernel
# trace: kernel families and GPU idle gaps of the timed steps
set -o pipefail
O=gpurun_out/r04/rank8
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o r8 -- python bench.py --steps 3 --warmup 1 --prompts 8 --no-cpu-baseline --out $O/bench.json > $O/bench.log 2>&1 || { echo "rocprof FAILED"; tail -20 $O/bench.log; exit 1; }
st=$(find $O/prof -name "*kernel_stats.csv" | head -1)
kt=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python tools/prof_summary.py $st > $O/summary.txt
python tools/trace_gaps.py $kt --window 0 --top 15 --timeline 300 > $O/gaps.txt
head -8 $O/summary.txt; cat $O/gaps.txt
rm -f $kt
