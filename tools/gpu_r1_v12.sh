#!/bin/bash
# GPU box: attention / actor tests, grouped-dkdv microbench, bench with 1 vs 2 log-prob streams.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 limit=$2; shift 2; timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; echo "[$name] rc=$rc"; return $rc; }
run tests_v12 600 python -u -m pytest tests/test_attention_gpu.py tests/test_actor_gpu.py tests/test_model_ops_gpu.py -m gpu -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread; rc=$?
if [ $rc -ge 2 ]; then exit $rc; fi
tail -3 gpurun_out/tests_v12.log
run attn64 300 python tools/model_microbench.py gfx950_n64 || exit $?
grep case gpurun_out/attn64.log
for ns in 1 2; do
  run bench_s$ns 400 python bench.py --steps 2 --warmup 1 --logprob-streams $ns --no-cpu-baseline || exit $?
  grep -E "^\{" gpurun_out/bench_s$ns.log | cut -c1-160
done
exit 0
