# round 4 evidence at HEAD: the headline bench line, the same command under rocprofv3 (kernel stats
# by family; the dominant kernels' averages must agree with the line's HIP-event timings), and the
# f1 forward's PMC traffic (FETCH_SIZE x2 + WRITE_SIZE, separate passes)
set -o pipefail
O=gpurun_out/r04
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --out $O/bench_g_headline.json > $O/bench_g_headline.log 2>&1 || { echo "bench FAILED"; tail -30 $O/bench_g_headline.log; exit 1; }
python -c "import json;d=json.load(open('$O/bench_g_headline.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline_hbm']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_g -o headline -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --out $O/bench_g_under_rocprof.json > $O/bench_g_prof.log 2>&1 || { echo "rocprof bench FAILED"; tail -30 $O/bench_g_prof.log; exit 1; }
st=$(find $O/prof_g -name "*kernel_stats.csv" | head -1)
python tools/prof_summary.py $st > $O/kernel_stats_headline_g_summary.txt
cp $st $O/kernel_stats_headline_g.csv
head -12 $O/kernel_stats_headline_g_summary.txt
find $O/prof_g -name "*kernel_trace.csv" -delete
timeout -k 10 600 bash tools/f1_pmc.sh > $O/f1_pmc.log 2>&1 || { echo "f1 pmc FAILED"; tail -20 $O/f1_pmc.log; exit 1; }
cp gpurun_out/f1pmc/summary.json $O/pmc_f1_product_r04.json
grep traffic_bytes_per_launch $O/pmc_f1_product_r04.json
