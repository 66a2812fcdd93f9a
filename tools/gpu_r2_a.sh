#!/bin/bash
# round 2: parity tests + smoke + N=1 bench + 2-rank gloo rehearsal of the launcher on one GPU
set -u
mkdir -p gpurun_out
run() { local name=$1 limit=$2; shift 2; timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; echo "[$name] rc=$rc"; return $rc; }
run tests 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
run smoke 300 python __graft_entry__.py smoke || exit $?
run bench 900 python bench.py --steps 3 --warmup 1 --out gpurun_out/bench.json || exit $?
VA_DIST_BACKEND=gloo run bench_w2_gloo 900 python bench.py --gpus 2 --steps 2 --warmup 1 --micro 32 --logprob-micro 32 --balance --out gpurun_out/bench_w2_gloo.json || exit $?
exit 0
