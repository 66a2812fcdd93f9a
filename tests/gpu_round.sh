#!/bin/bash
# One GPU session: parity tests, smoke, then the benchmark. Every GPU step has its own time
# limit and a fault (rc >= 2 from pytest, or any signal exit) stops the script.
set -u
mkdir -p gpurun_out
STAGE=${1:-all}
run() { local name=$1 limit=$2; shift 2; timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; echo "[$name] rc=$rc"; return $rc; }
if [[ $STAGE == all || $STAGE == tests ]]; then
  run tests 900 python -m pytest tests -m gpu -q -rf -p no:cacheprovider; rc=$?
  if [ $rc -ge 2 ]; then exit $rc; fi
  run smoke 300 python __graft_entry__.py smoke || exit $?
fi
if [[ $STAGE == all || $STAGE == bench ]]; then
  run bench_small 400 python bench.py --prompts 8 --steps 2 --warmup 1 --no-cpu-baseline || exit $?
  run bench 900 python bench.py --steps 3 --warmup 1 --out gpurun_out/bench.json || exit $?
fi

if [[ $STAGE == prof ]]; then
  export TMPDIR=/tmp
  run prof_small 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_small -o run -- python bench.py --prompts 8 --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing || exit $?
fi
if [[ $STAGE == kbench ]]; then
  export TMPDIR=/tmp
  run kbench 600 python tools/kernel_bench.py || exit $?
  run kb_trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kb_trace -o run -- python tools/kernel_bench.py --only logprob --iters 10 || exit $?
  run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python tools/kernel_bench.py --only logprob --iters 5 || exit $?
  run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python tools/kernel_bench.py --only logprob --iters 5 || exit $?
fi
if [[ $STAGE == dp ]]; then
  run tests_dp 600 python -m pytest tests/test_dp_gpu.py -q -rf -p no:cacheprovider; rc=$?
  if [ $rc -ge 2 ]; then exit $rc; fi
fi
if [[ $STAGE == sweep ]]; then
  export TMPDIR=/tmp
  run sweep8k 600 python tools/kernel_bench.py --sweep --rows 8192 || exit $?
  run sweep16k 600 python tools/kernel_bench.py --sweep --rows 16384 || exit $?
  run small_trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/small_trace -o run -- python tools/kernel_bench.py --only small --iters 10 || exit $?
fi
exit 0
