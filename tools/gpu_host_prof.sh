#!/bin/bash
# host-side cProfile of the timed steps at the N = 8 per-rank workload (8 prompts, world 1)
set -u
O=gpurun_out/hostprof
mkdir -p $O
VA_BENCH_CPROFILE=$O/p8.prof timeout -k 10 300 python bench.py --prompts 8 --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-timing --out $O/p8.json > $O/p8.log 2>&1 || exit $?
python3 - <<'PY'
import pstats
p = pstats.Stats("gpurun_out/hostprof/p8.prof")
p.sort_stats("tottime").print_stats(30)
p.sort_stats("cumulative").print_stats(40)
PY
