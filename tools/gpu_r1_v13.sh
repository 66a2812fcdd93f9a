#!/bin/bash
# GPU box: model-side tests (attention, model ops, actor), then the headline bench.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-v13}
run() { local name=$1 limit=$2; shift 2; timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; echo "[$name] rc=$rc"; return $rc; }
run tests_$TAG 600 python -u -m pytest tests/test_attention_gpu.py tests/test_model_ops_gpu.py tests/test_actor_gpu.py -m gpu -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread; rc=$?
tail -15 gpurun_out/tests_$TAG.log | grep -v "^W20"
if [ $rc -ne 0 ]; then exit $rc; fi
run bench_$TAG 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline || exit $?
grep -E "^\{" gpurun_out/bench_$TAG.log | cut -c1-160
exit 0
