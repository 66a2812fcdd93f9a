# round 5 GPU pass h: the headline at HEAD — bench.py as the driver runs it (with the CPU baseline),
# the same command under rocprofv3 --kernel-trace --stats (kernel families, per-step idle of the timed
# steps), and the f1 HBM traffic PMC passes (FETCH_SIZE x2 + WRITE_SIZE)
set -o pipefail
O=gpurun_out/r05/h
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 python bench.py --out $O/bench_headline.json > $O/bench_headline.log 2>&1 || { echo "bench FAILED"; tail -30 $O/bench_headline.log; exit 1; }
python -c "import json;d=json.load(open('$O/bench_headline.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline_hbm']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o headline -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --out $O/bench_under_rocprof.json > $O/bench_prof.log 2>&1 || { echo "rocprof bench FAILED"; tail -30 $O/bench_prof.log; exit 1; }
st=$(find $O/prof -name "*kernel_stats.csv" | head -1)
kt=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python tools/prof_summary.py $st > $O/kernel_stats_headline_summary.txt
cp $st $O/kernel_stats_headline.csv
python tools/trace_gaps.py $kt --steps 3 --top 12 | tail -16 > $O/trace_gaps_headline.txt
python tools/prof_split.py $kt > $O/kernels_by_grid.txt 2>/dev/null || true
head -14 $O/kernel_stats_headline_summary.txt; cat $O/trace_gaps_headline.txt | head -5
gzip -c $kt > $O/kernel_trace_headline.csv.gz && rm -f $kt
timeout -k 10 600 bash tools/f1_pmc.sh > $O/f1_pmc.log 2>&1 || { echo "f1 pmc FAILED"; tail -20 $O/f1_pmc.log; exit 1; }
cp gpurun_out/f1pmc/summary.json $O/pmc_f1_product.json
grep traffic_bytes_per_launch $O/pmc_f1_product.json
