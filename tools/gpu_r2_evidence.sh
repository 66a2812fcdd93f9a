#!/bin/bash
# round 2 evidence in one GPU call: log-prob PMC traffic + stream ceilings at the bench launch,
# full GPU tests, smoke, headline bench (N=1, CPU baseline), rocprofv3 stats of the bench,
# small-kernel device times + PMC traffic at 512 / 8,192 rows.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2ev
mkdir -p $O
export TMPDIR=/tmp
ROWS=131072
TAG=${1:-v2}
run() { local name=$1 limit=$2; shift 2; timeout -k 10 "$limit" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "$O/$name.log"; echo "[$name] rc=$rc"; return $rc; }
if [[ ${PMC:-1} == 1 ]]; then
  hipcc -O3 --offload-arch=gfx950 -o $O/hbm_stream tools/hbm_stream.hip || exit 1
  run hbm_$ROWS 300 $O/hbm_stream $ROWS || exit $?
  grep -E "^\{" $O/hbm_$ROWS.log > $O/hbm_stream_${ROWS}rows.jsonl
  rm -f $O/hbm_stream
  run pmc_fetch_lp 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_lp -o run -- python3 tools/kernel_bench.py --only logprob --rows $ROWS --iters 3 || exit $?
  run pmc_write_lp 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_lp -o run -- python3 tools/kernel_bench.py --only logprob --rows $ROWS --iters 3 || exit $?
  python3 tools/pmc_summary.py $O/pmc_fetch_lp $O/pmc_write_lp $ROWS 151936 $O/pmc_logprob_${ROWS}rows.json > /dev/null || exit 1
  run pmc_fetch_small 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_small -o run -- python3 tools/small_kernels_bench.py --iters 5 || exit $?
  run pmc_write_small 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_small -o run -- python3 tools/small_kernels_bench.py --iters 5 || exit $?
  python3 tools/pmc_split.py $O/pmc_fetch_small $O/pmc_write_small --match va:: > $O/pmc_small_kernels.jsonl || exit 1
  find $O -name "*.db" -delete
  find $O/pmc_* -name "*.csv" ! -name "*counter_collection.csv" -delete
fi
if [[ ${TESTS:-1} == 1 ]]; then
  run tests_$TAG 900 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 300 --timeout-method thread; rc=$?
  tail -3 $O/tests_$TAG.log
  if [ $rc -ge 2 ]; then exit $rc; fi
  run smoke_$TAG 300 python __graft_entry__.py smoke || exit $?
fi
run small_$TAG 300 python tools/small_kernels_bench.py || exit $?
run prof_small_$TAG 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_small_$TAG -o run -- python tools/small_kernels_bench.py || exit $?
python3 tools/prof_split.py $O/prof_small_$TAG/run_kernel_trace.csv --match va:: > $O/prof_small_$TAG.split.jsonl || true
if [[ ${BENCH:-1} == 0 ]]; then exit 0; fi
run bench_$TAG 900 python bench.py --steps 3 --warmup 1 --out $O/bench_$TAG.json || exit $?
run prof_$TAG 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 --out $O/bench_prof_$TAG.json || exit $?
f=$(find $O/prof_$TAG -name '*kernel_stats.csv' | head -1)
python3 tools/prof_summary.py "$f" > $O/prof_$TAG.summary.txt && cp "$f" $O/prof_$TAG.kernel_stats.csv
t=$(find $O/prof_$TAG -name '*kernel_trace.csv' | head -1)
python3 tools/trace_gaps.py "$t" --window 3.0 > $O/prof_$TAG.gaps.txt || true
find $O/prof_$TAG $O/prof_small_$TAG \( -name "*kernel_trace.csv" -o -name "*.db" \) -delete
exit 0
