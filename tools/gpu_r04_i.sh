# NOTE: records the run at commit 44487f4; the ring variant was removed after it and tuning key 19 is
# now VA_TUNE_FLASH_DMA, so rerun this script only at that commit.
# f1 forward: the deep-ring variant (VA_TUNE_F1_RING = 19: 0 two 64-deep buffers, 4 / 5 ring stages of
# 32) interleaved, with its deviation from the unfused path (must stay 0 / within 2e-6), then SQ
# counters of each (MFMA busy, waits, clock)
set -o pipefail
O=gpurun_out/r04/f1_ring
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for r in 1 2; do
  for ring in 0 4 5; do
    timeout -k 10 120 python tools/f1_ab.py --tag ring$ring --tune 19=$ring >> $O/time.jsonl 2>>$O/err.log || { echo "f1_ab ring$ring FAILED"; tail $O/err.log; exit 1; }
  done
done
python -c "
import json
for l in open('$O/time.jsonl'):
    d=json.loads(l); print(d['tag'], d['ms_median'], d['tflops'], d['max_dlp_vs_unfused'], d['max_dent_vs_unfused'])"
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE"
for ring in 0 4; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/sq$ring -o run -- python3 tools/f1_ab.py --iters 1 --tune 19=$ring > $O/sq$ring.log 2>&1 || { echo "sq $ring FAILED"; tail $O/sq$ring.log; exit 1; }
  python3 - $ring <<'PY'
import csv, glob, sys, collections
ring = sys.argv[1]
d = f"gpurun_out/r04/f1_ring/sq{ring}"
cc = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
kt = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
per = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(cc)):
    if "linear_logprob_t256_kernel" in r["Kernel_Name"]:
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
dur = {}
for r in csv.DictReader(open(kt)):
    if "linear_logprob_t256_kernel" in r["Kernel_Name"]:
        dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
did = max(per, key=lambda k: per[k]["GRBM_GUI_ACTIVE"])
v = per[did]
wc = v["SQ_WAVE_CYCLES"] or 1
ms = dur.get(did, 0) / 1e6
clock = v["GRBM_GUI_ACTIVE"] / 8 / dur[did] if dur.get(did) else float("nan")
busy = v["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * v["GRBM_GUI_ACTIVE"] / 8)
print(f"ring {ring}: {ms:.2f} ms, mfma busy {busy:.3f}, clock {clock:.2f} GHz, busy x clock {busy * clock:.3f}, "
      f"wait_any {v['SQ_WAIT_ANY'] / wc:.3f}, active_inst {v['SQ_ACTIVE_INST_ANY'] / wc:.3f}")
PY
  find $O/sq$ring -name "*.csv" -size +2M -delete
done | tee $O/sq_summary.txt
