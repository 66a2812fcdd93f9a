#!/bin/bash
# GPU box: rocprofv3 kernel-trace stats of one headline bench step (after 1 warmup).
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out "$(dirname "gpurun_out/${1:-prof_bench}")"
OUT=${1:-prof_bench}
shift
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$OUT -o run -- python3 bench.py --no-cpu-baseline --no-kernel-timing --steps 1 --warmup 1 "$@" > gpurun_out/$OUT.log 2>&1
echo "[prof] rc=$?"
grep -v "^W20" gpurun_out/$OUT.log | tail -15; find gpurun_out/$OUT | head
f=$(find gpurun_out/$OUT -name '*kernel_stats.csv' | head -1)
python3 tools/prof_summary.py "$f" > gpurun_out/$OUT.summary.txt && cp "$f" gpurun_out/$OUT.kernel_stats.csv
find gpurun_out/$OUT \( -name "*kernel_trace.csv" -o -name "*.db" \) -delete
head -60 gpurun_out/$OUT.summary.txt
