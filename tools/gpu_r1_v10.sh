#!/bin/bash
# GPU box: full GPU tests, smoke, headline bench (defaults), HBM calibration + log-prob kernels at
# the 65,536-row micro-batch.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-v10}
run() { local name=$1 limit=$2; shift 2; timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; echo "[$name] rc=$rc"; return $rc; }
run tests_$TAG 900 python -u -m pytest tests -m gpu -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread; rc=$?
if [ $rc -ge 2 ]; then exit $rc; fi
tail -3 gpurun_out/tests_$TAG.log
run smoke_$TAG 300 python __graft_entry__.py smoke || exit $?
run bench_$TAG 900 python bench.py --steps 3 --warmup 1 --out gpurun_out/bench_$TAG.json || exit $?
grep -E "^\{" gpurun_out/bench_$TAG.log | cut -c1-200
hipcc -O3 --offload-arch=gfx950 -o gpurun_out/hbm_stream tools/hbm_stream.hip || exit 1
run hbm65k 300 gpurun_out/hbm_stream 65536 || exit $?
rm -f gpurun_out/hbm_stream
run kb65k 300 python tools/kernel_bench.py --only logprob --rows 65536 --iters 5 || exit $?
grep kernel gpurun_out/kb65k.log
exit 0
