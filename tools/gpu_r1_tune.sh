#!/bin/bash
# GPU box: padding parity tests, then the offline GEMM search (tools/tune_gemms.py) and a bench
# with / without the resulting table. Stops at the first timeout / fault.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 limit=$2; shift 2; timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; echo "[$name] rc=$rc"; return $rc; }
run tests_pad 300 python -u -m pytest tests/test_actor_gpu.py -m gpu -q -rf -p no:cacheprovider --timeout 120 --timeout-method thread -k pack_pad; rc=$?
if [ $rc -ge 2 ]; then exit $rc; fi
TABLE=gpurun_out/gemm_table.csv
PYTORCH_TUNABLEOP_VERBOSE=1 run tune ${TUNE_LIMIT:-780} python -u tools/tune_gemms.py --out $TABLE --seeds ${SEEDS:-4} --micro ${MICRO:-64} --logprob-micro ${MICRO:-64} --pad ${PAD:-2048} || exit $?
grep -c "^Gemm" $TABLE
grep "^\[tune" gpurun_out/tune.log | tail -3
run bench_tuned 400 python bench.py --steps 2 --warmup 1 --micro ${MICRO:-64} --logprob-micro ${MICRO:-64} --pad-multiple ${PAD:-2048} --gemm-table $TABLE --no-cpu-baseline || exit $?
grep -E "^\{" gpurun_out/bench_tuned.log | cut -c1-200
exit 0
