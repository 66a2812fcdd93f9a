#!/bin/bash
# small-kernel device times (rocprofv3 kernel trace split per launch shape) + wall times; extra args go to the bench
set -u
O=gpurun_out/small
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/small_kernels_bench.py "$@" > $O/wall.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python tools/small_kernels_bench.py "$@" > $O/prof.log 2>&1 || exit $?
python3 tools/prof_split.py $O/prof/run_kernel_trace.csv --match va:: --phases ${PHASES:-1} > $O/split.jsonl
rm -f $O/prof/run_kernel_trace.csv
grep '"op"' $O/wall.log; cat $O/split.jsonl
