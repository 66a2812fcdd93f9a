# f1 forward: weight re-fetch vs time. The vocab ranges per row block (splits) set how many row
# blocks share each streamed weight tile in an XCD's L2 (32 resident workgroups = 32/splits row
# blocks x splits ranges): fewer splits, less fabric traffic. Time and FETCH_SIZE per setting.
set -o pipefail
O=gpurun_out/r04/f1_splits
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for sp in 8 4 2 16 8; do
  VERL_AMD_LINEAR_LOGPROB_SPLITS=$sp timeout -k 10 120 python tools/f1_ab.py --tag splits$sp >> $O/time.jsonl 2>>$O/err.log || { echo "f1_ab $sp FAILED"; tail $O/err.log; exit 1; }
done
cat $O/time.jsonl | python -c "import sys,json; [print(json.loads(l)['tag'], json.loads(l)['ms_median'], json.loads(l)['tflops']) for l in sys.stdin]"
for sp in 8 4 2; do
  VERL_AMD_LINEAR_LOGPROB_SPLITS=$sp timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch$sp -o run -- python3 tools/f1_ab.py --iters 2 > $O/fetch$sp.log 2>&1 || { echo "pmc $sp FAILED"; tail $O/fetch$sp.log; exit 1; }
  python3 - $sp <<'PY'
import csv, glob, statistics, sys
sp = sys.argv[1]
p = glob.glob(f"gpurun_out/r04/f1_splits/fetch{sp}/**/*counter_collection.csv", recursive=True)[0]
per = {}
for r in csv.DictReader(open(p)):
    if "linear_logprob_t256_kernel" in r["Kernel_Name"] and r["Counter_Name"].startswith("FETCH_SIZE"):
        per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
v = statistics.median(sorted(per.values()))
print(f"splits {sp}: fetch x2 {v * 1024 * 2 / 1e9:.1f} GB per launch ({len(per)} launches)")
PY
  find $O/fetch$sp -name "*.csv" -size +2M -delete
done | tee $O/fetch_summary.txt
