#!/bin/bash
# GPU box: GEMM table for 128-response micro-batches, then bench m64 (committed table) vs m128.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 limit=$2; shift 2; timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; echo "[$name] rc=$rc"; return $rc; }
cp verl_amd/tuned/gemm_qwen2_0p5b_mi355x.csv gpurun_out/table128.csv
PYTORCH_TUNABLEOP_VERBOSE=1 run tune128 700 python -u tools/tune_gemms.py --out gpurun_out/table128.csv --seeds 2 --micro 128 --logprob-micro 128 --pad 2048 || exit $?
grep "^\[tune" gpurun_out/tune128.log | tail -2
run b64 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline || exit $?
grep -E "^\{" gpurun_out/b64.log | cut -c60-130
run b128 500 python bench.py --steps 2 --warmup 1 --micro 128 --logprob-micro 128 --gemm-table gpurun_out/table128.csv --no-cpu-baseline || exit $?
grep -E "^\{" gpurun_out/b128.log | cut -c60-130
grep -o '"peak_hbm_gb": [0-9.]*' gpurun_out/b128.log
exit 0
