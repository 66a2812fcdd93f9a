# round 5 GPU pass aq: the no-grad pass with the fused lm_head (f1, default) vs the unfused
# hipBLASLt lm_head GEMM + streaming log-prob forward (--fused-no-grad 0), interleaved at the final head
set -o pipefail
O=gpurun_out/r05/aq
mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 400 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --out $O/bench_$tag.json "$@" > $O/bench_$tag.log 2>&1 || { echo "$tag FAILED"; tail -20 $O/bench_$tag.log; exit 1; }; python -c "import json;d=json.load(open('$O/bench_$tag.json'));print('$tag', d['value'], d['ms_per_step'])"; }
run fused_1
run unfused_1 --fused-no-grad 0
run fused_2
run unfused_2 --fused-no-grad 0
