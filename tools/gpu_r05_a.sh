# round 5 GPU pass a: this round's baselines at HEAD — the full-batch headline, the N = 8 per-rank
# workload (8 prompts) with a torch op profile of its timed steps (where the small launches come
# from), and the same workload under a kernel trace (per-step GPU idle, gaps by kernel pair)
set -o pipefail
O=gpurun_out/r05/a
mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu-baseline --out $O/full.json > $O/full.log 2>&1 || { echo "full FAILED"; tail -20 $O/full.log; exit 1; }
python -c "import json;d=json.load(open('$O/full.json'));print('full', d['value'], d['ms_per_step'], d['roofline']['frac'])"
VA_BENCH_TORCH_PROFILE=$O/p8_torchprof.txt timeout -k 10 300 python bench.py --prompts 8 --no-cpu-baseline --out $O/p8_prof.json > $O/p8_prof.log 2>&1 || { echo "p8 prof FAILED"; tail -20 $O/p8_prof.log; exit 1; }
python -c "import json;d=json.load(open('$O/p8_prof.json'));print('p8 (torch profiler on)', d['value'], d['ms_per_step'])"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p8 -- python bench.py --steps 3 --warmup 1 --prompts 8 --no-cpu-baseline --out $O/p8_trace.json > $O/p8_trace.log 2>&1 || { echo "rocprof FAILED"; tail -20 $O/p8_trace.log; exit 1; }
st=$(find $O/prof -name "*kernel_stats.csv" | head -1)
kt=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python tools/prof_summary.py $st > $O/p8_summary.txt
python tools/trace_gaps.py $kt --steps 3 --top 40 > $O/p8_gaps.txt
cat $O/p8_gaps.txt | head -50
gzip -c $kt > $O/p8_kernel_trace.csv.gz && rm -f $kt
