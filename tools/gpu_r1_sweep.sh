#!/bin/bash
# GPU box: PMC HBM-traffic passes for the log-prob kernels + a micro-batch sweep of the bench.
# Python errors (rc=1, e.g. OOM) continue; timeouts / signals / faults stop the script.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 limit=$2; shift 2; timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; echo "[$name] rc=$rc"; return $rc; }
ok() { [ "$1" -le 1 ]; }
if [[ ${PMC:-1} == 1 ]]; then
run pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 tools/kernel_bench.py --only logprob --iters 5 || exit $?
run pmc_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 tools/kernel_bench.py --only logprob --iters 5 || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write 8192 151936 gpurun_out/pmc_logprob.json
find gpurun_out/pmc_fetch gpurun_out/pmc_write -name "*.db" -delete
fi
for cfg in ${SWEEP:-"16 32" "32 32" "16 64"}; do
  set -- $cfg
  run bench_m$1_l$2 400 python bench.py --steps 2 --warmup 1 --micro $1 --logprob-micro $2 --no-cpu-baseline; rc=$?
  ok $rc || exit $rc
  grep -E "^\{" gpurun_out/bench_m$1_l$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('micro', $1, $2, d['value'], d['ms_per_step'])" || true
done
exit 0
