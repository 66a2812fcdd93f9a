# round 5 GPU pass b: the vocab-split fused lm_head backward (ABI 6) and the non-blocking step
# boundary (host mask mirror + asynchronous metric readback) — full GPU suite, the range-width
# A/B at the bench's 131,072-row pass, bench with --fused-kernels 1 (peak HBM) next to the default,
# the 196,608-token dynamic budget under --fused-kernels 1, and the 8-prompt per-rank workload
# under a kernel trace (per-step idle)
set -o pipefail
O=gpurun_out/r05/b
mkdir -p $O
export VA_REHEARSAL_OUT=$O/rehearsal
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest FAILED"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python tools/f1_bwd_ab.py --iters 3 --vocab-splits 9504,19008,37984,75968 > $O/f1_bwd_splits.jsonl 2> $O/f1_bwd_splits.err || { echo "f1_bwd_ab FAILED"; tail -20 $O/f1_bwd_splits.err; exit 1; }
cat $O/f1_bwd_splits.jsonl
timeout -k 10 300 python bench.py --no-cpu-baseline --fused-kernels 1 --out $O/bench_fused.json > $O/bench_fused.log 2>&1 || { echo "bench fused FAILED"; tail -20 $O/bench_fused.log; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --out $O/bench_default.json > $O/bench_default.log 2>&1 || { echo "bench default FAILED"; tail -20 $O/bench_default.log; exit 1; }
for f in bench_fused bench_default; do python -c "import json;d=json.load(open('$O/$f.json'));print('$f', d['value'], d['ms_per_step'], d['config']['peak_hbm_gb'], d['clip_branch_tokens_timed_steps'], d['final_metrics'].get('perf/mfu/actor'))"; done
timeout -k 10 500 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --fused-kernels 1 --responses realistic --dynamic-bsz 196608 --out $O/bench_fused_dyn196608.json > $O/bench_fused_dyn196608.log 2>&1 || { echo "bench dyn196608 FAILED"; tail -30 $O/bench_fused_dyn196608.log; exit 1; }
python -c "import json;d=json.load(open('$O/bench_fused_dyn196608.json'));print('dyn196608 fused', d['value'], d['ms_per_step'], d['config']['peak_hbm_gb'], d['config']['logprob_bwd_inplace_fallbacks'])"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p8 -- python bench.py --steps 3 --warmup 1 --prompts 8 --no-cpu-baseline --out $O/p8_trace.json > $O/p8_trace.log 2>&1 || { echo "rocprof FAILED"; tail -20 $O/p8_trace.log; exit 1; }
kt=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python tools/trace_gaps.py $kt --steps 3 --top 12 | tail -16 > $O/p8_gaps.txt
cat $O/p8_gaps.txt
python -c "import json;d=json.load(open('$O/p8_trace.json'));print('p8 traced', d['value'], d['ms_per_step'])"
rm -f $kt
