#!/bin/bash
# GPU box: evidence at the bench's own log-prob launch size (micro-batch 128 -> 131,072 response
# rows per launch): PMC HBM traffic of the log-prob kernels, plain-stream ceilings at the same
# footprint, then tests / smoke / bench / rocprofv3 stats of the bench command (gpu_r1_final.sh).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
ROWS=${ROWS:-131072}
run() { local name=$1 limit=$2; shift 2; timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc" >> "gpurun_out/$name.log"; echo "[$name] rc=$rc"; return $rc; }
hipcc -O3 --offload-arch=gfx950 -o gpurun_out/hbm_stream tools/hbm_stream.hip || exit 1
run hbm_$ROWS 300 gpurun_out/hbm_stream $ROWS || exit $?
grep -E "^\{" gpurun_out/hbm_$ROWS.log > gpurun_out/hbm_stream_${ROWS}rows.jsonl
rm -f gpurun_out/hbm_stream
run kb_$ROWS 300 python3 tools/kernel_bench.py --only logprob --rows $ROWS --iters 5 || exit $?
run pmc_fetch_$ROWS 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_$ROWS -o run -- python3 tools/kernel_bench.py --only logprob --rows $ROWS --iters 3 || exit $?
run pmc_write_$ROWS 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_$ROWS -o run -- python3 tools/kernel_bench.py --only logprob --rows $ROWS --iters 3 || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc_fetch_$ROWS gpurun_out/pmc_write_$ROWS $ROWS 151936 gpurun_out/pmc_logprob_${ROWS}rows.json || exit 1
find gpurun_out/pmc_fetch_$ROWS gpurun_out/pmc_write_$ROWS -name "*.db" -delete
mkdir -p profiles/r01 && cp gpurun_out/pmc_logprob_${ROWS}rows.json gpurun_out/hbm_stream_${ROWS}rows.jsonl profiles/r01/
exec_final=${FINAL:-1}
if [[ $exec_final == 1 ]]; then
  bash tools/gpu_r1_final.sh ${TAG:-v15}
fi
