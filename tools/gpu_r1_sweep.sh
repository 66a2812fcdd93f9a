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
IFS=',' read -ra CFGS <<< "${SWEEP:-16 32 0,32 32 0}"
for cfg in "${CFGS[@]}"; do
  set -- $cfg
  n=bench_m$1_l$2_d$3
  run $n 400 python bench.py --steps 2 --warmup 1 --micro $1 --logprob-micro $2 --dynamic-bsz $3 --no-cpu-baseline; rc=$?
  ok $rc || exit $rc
  grep -E "^\{" gpurun_out/$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['ms_per_step'], d['config']['peak_hbm_gb'])" || true
done
if [[ -n ${TUNE_T:-} ]]; then
  run tunableop 600 python tools/tunableop_probe.py $TUNE_T || exit $?
  cat gpurun_out/tunableop.log
fi
exit 0
