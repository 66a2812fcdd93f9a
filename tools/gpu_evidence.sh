#!/bin/bash
# GPU box, one call: the whole -m gpu suite (one process), smoke(), the default bench line, and the
# same bench command under rocprofv3 --kernel-trace --stats (its summary is what profiles/ keeps).
# $1 = tag for the output names.
set -u
T=${1:-ev}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_gpu_$T.log 2>&1
rc=$?; echo "[pytest -m gpu] rc=$rc"; tail -3 gpurun_out/pytest_gpu_$T.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1
rc=$?; echo "[smoke] rc=$rc"; tail -2 gpurun_out/smoke_$T.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; echo "[bench] rc=$rc"; tail -c 400 gpurun_out/bench_$T.json
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$T -o run -- \
  python3 bench.py > gpurun_out/bench_under_rocprof_$T.json 2> gpurun_out/bench_under_rocprof_$T.err
rc=$?; echo "[rocprof bench] rc=$rc"
[ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/prof_$T -name '*kernel_stats.csv' | head -1)
python3 tools/prof_summary.py "$f" > gpurun_out/kernel_stats_$T.summary.txt && cp "$f" gpurun_out/kernel_stats_$T.csv
find gpurun_out/prof_$T \( -name "*kernel_trace.csv" -o -name "*.db" \) -delete
head -30 gpurun_out/kernel_stats_$T.summary.txt
