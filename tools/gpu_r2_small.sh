#!/bin/bash
# round 2: core-algos kernels — parity tests, wall-time microbench, rocprof device times
set -u
mkdir -p gpurun_out/r2small
export TMPDIR=/tmp
run() { local name=$1 limit=$2; shift 2; timeout -k 10 "$limit" "$@" > "gpurun_out/r2small/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/r2small/$name.log"; echo "[$name] rc=$rc"; return $rc; }
run tests 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider -k "gae or grpo or outcome or whiten or dp_adv or estimators or loss or custom_ops" || exit $?
for cfg in ${CFGS:-1:0 1:3 1:7 4:3}; do
  P=${cfg%%:*}; NT=${cfg##*:}
  run wall_p${P}_nt$NT 300 python tools/small_kernels_bench.py --gae-partials $P --gae-nt $NT || exit $?
  run prof_p${P}_nt$NT 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2small/prof_p${P}_nt$NT -o run -- python tools/small_kernels_bench.py --gae-partials $P --gae-nt $NT || exit $?
done
exit 0
