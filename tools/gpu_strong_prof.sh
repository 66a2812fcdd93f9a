#!/bin/bash
# rocprofv3 kernel stats of the N = 8 per-rank workload (8 prompts x 8 responses, world 1)
set -u
O=gpurun_out/strongprof
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p8 -o run -- python3 bench.py --prompts 8 --steps 2 --warmup 1 --no-cpu-baseline --out $O/p8.json > $O/p8.log 2>&1 || exit $?
f=$(find $O/p8 -name '*kernel_stats.csv' | head -1)
python3 tools/prof_summary.py "$f" > $O/p8.summary.txt
t=$(find $O/p8 -name '*kernel_trace.csv' | head -1)
python3 tools/trace_gaps.py "$t" --window 0.74 > $O/p8.gaps.txt || true
find $O/p8 \( -name "*kernel_trace.csv" -o -name "*.db" \) -delete
