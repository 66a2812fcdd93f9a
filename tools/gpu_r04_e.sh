# round 4 GPU pass e: the realistic variant at the 196,608-token dynamic budget that ran out of memory
# in round 3 with the out-of-place log-prob backward; now "auto" falls back in place when the dlogits
# buffer does not fit
set -o pipefail
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 500 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --responses realistic --dynamic-bsz 196608 --out $O/bench_e_dyn196608.json > $O/bench_e_dyn196608.log 2>&1 || { echo "bench dyn196608 FAILED"; tail -30 $O/bench_e_dyn196608.log; exit 1; }
python -c "import json;d=json.load(open('$O/bench_e_dyn196608.json'));print(d['value'], d['ms_per_step'], d['config']['peak_hbm_gb'], d['config']['logprob_bwd_inplace_fallbacks'])"
