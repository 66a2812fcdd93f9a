#!/bin/bash
# GPU box, round-end evidence in one call: full GPU tests, smoke, headline bench with the CPU
# baseline, rocprofv3 kernel stats + idle-gap analysis of the same bench command.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-final}
run() { local name=$1 limit=$2; shift 2; timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; echo "[$name] rc=$rc"; return $rc; }
run tests_$TAG 900 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread; rc=$?
tail -3 gpurun_out/tests_$TAG.log
if [ $rc -ge 2 ]; then exit $rc; fi
run smoke_$TAG 300 python __graft_entry__.py smoke || exit $?
run bench_$TAG 900 python bench.py --steps 3 --warmup 1 --out gpurun_out/bench_$TAG.json || exit $?
grep -E "^\{" gpurun_out/bench_$TAG.log | cut -c1-200
run prof_$TAG 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 --out gpurun_out/bench_prof_$TAG.json || exit $?
f=$(find gpurun_out/prof_$TAG -name '*kernel_stats.csv' | head -1)
python3 tools/prof_summary.py "$f" > gpurun_out/prof_$TAG.summary.txt && cp "$f" gpurun_out/prof_$TAG.kernel_stats.csv
t=$(find gpurun_out/prof_$TAG -name '*kernel_trace.csv' | head -1)
python3 tools/trace_gaps.py "$t" --window 3.0 > gpurun_out/prof_$TAG.gaps.txt || true
find gpurun_out/prof_$TAG \( -name "*kernel_trace.csv" -o -name "*.db" \) -delete
head -12 gpurun_out/prof_$TAG.summary.txt
exit 0
