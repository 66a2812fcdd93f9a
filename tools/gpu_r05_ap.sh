# round 5 GPU pass ap (= af at the final head): at HEAD after the f1 staging rework (buffer-resource LDS-DMA between the
# K-halves) and the fused gate|up + SwiGLU on by default — full GPU suite + smoke(), the headline
# bench as the driver runs it, the same under rocprofv3 --kernel-trace --stats, the f1 HBM traffic
# PMC passes, the 8-prompt per-rank workload, the fused lm_head forward + backward at pass level
set -o pipefail
O=gpurun_out/r05/ap
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export VA_REHEARSAL_OUT=$O/rehearsal
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest FAILED"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke FAILED"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --out $O/bench_headline.json > $O/bench_headline.log 2>&1 || { echo "bench FAILED"; tail -30 $O/bench_headline.log; exit 1; }
python -c "import json;d=json.load(open('$O/bench_headline.json'));r=d['roofline'];print('headline', d['value'], d['ms_per_step'], r['kernel'], r['frac'], r.get('launch_us_min_median_max'), d['roofline_hbm']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 400 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --prompts 8 --out $O/bench_p8.json > $O/bench_p8.log 2>&1 || { echo "p8 FAILED"; tail -30 $O/bench_p8.log; exit 1; }
python -c "import json;d=json.load(open('$O/bench_p8.json'));print('p8', d['value'], d['ms_per_step'])"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o headline -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --out $O/bench_under_rocprof.json > $O/bench_prof.log 2>&1 || { echo "rocprof bench FAILED"; tail -30 $O/bench_prof.log; exit 1; }
st=$(find $O/prof -name "*kernel_stats.csv" | head -1)
kt=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python tools/prof_summary.py $st > $O/kernel_stats_headline_summary.txt
cp $st $O/kernel_stats_headline.csv
python tools/trace_gaps.py $kt --steps 3 --top 12 | tail -16 > $O/trace_gaps_headline.txt
head -12 $O/kernel_stats_headline_summary.txt; grep "last 3" $O/trace_gaps_headline.txt
gzip -c $kt > $O/kernel_trace_headline.csv.gz && rm -f $kt
timeout -k 10 600 bash tools/f1_pmc.sh > $O/f1_pmc.log 2>&1 || { echo "f1 pmc FAILED"; tail -20 $O/f1_pmc.log; exit 1; }
cp gpurun_out/f1pmc/summary.json $O/pmc_f1_product.json
grep traffic_bytes_per_launch $O/pmc_f1_product.json
timeout -k 10 400 python tools/f1_bwd_ab.py > $O/f1_bwd_ab.jsonl 2> $O/f1_bwd_ab.err || { echo "f1 bwd FAILED"; tail -20 $O/f1_bwd_ab.err; exit 1; }
tail -3 $O/f1_bwd_ab.jsonl
