#!/bin/bash
# GPU box: rocprofv3 kernel stats of one bench step for a given bench config (+ wgrad microbench).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
run() { local name=$1 limit=$2; shift 2; timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; echo "[$name] rc=$rc"; return $rc; }
if [[ -n ${WGRAD_T:-} ]]; then run wgrad 300 python tools/wgrad_bench.py $WGRAD_T || exit $?; cat gpurun_out/wgrad.log | grep case; fi
run prof_$TAG 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 --out gpurun_out/bench_prof_$TAG.json "$@" || exit $?
f=$(find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1)
python3 tools/prof_summary.py "$f" > gpurun_out/prof_$TAG.summary.txt && cp "$f" gpurun_out/prof_$TAG.kernel_stats.csv
t=$(find gpurun_out/prof_$TAG -name '*kernel_trace.csv' | head -1)
python3 tools/trace_gaps.py "$t" --window ${GAP_WINDOW:-3.0} > gpurun_out/prof_$TAG.gaps.txt || true
find gpurun_out/prof_$TAG \( -name "*kernel_trace.csv" -o -name "*.db" \) -delete
head -8 gpurun_out/prof_$TAG.summary.txt
exit 0
