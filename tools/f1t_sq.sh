#!/bin/bash
# SQ / GRBM counters of the f1 dev kernels at 131,072 x 896 x 151,936 (8 vocab ranges): MFMA-pipe
# busy share, wave wait / issue-stall / active shares, and the effective clock (GRBM_GUI_ACTIVE / 8
# XCDs / kernel time). Variants as tools/f1t_bench.py (0 core only + remap, 1 full + remap).
#   tools/f1t_sq.sh 0 1
set -u
O=gpurun_out/f1tsq
mkdir -p $O
export TMPDIR=/tmp
V="${*:-0 1}"
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/sq -o run -- python3 tools/f1t_bench.py --rows 131072 --splits 8 --variants $V --iters 1 --no-product > $O/sq.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob, collections, json
p = glob.glob("gpurun_out/f1tsq/sq/**/*counter_collection.csv", recursive=True)[0]
rows = list(csv.DictReader(open(p)))
per = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    n = r["Kernel_Name"]
    if "lp_" not in n and "Cijk" not in n:
        continue
    key = (n[:72], r.get("Grid_Size", ""), r.get("Dispatch_Id", ""))
    per[key][r["Counter_Name"]] += float(r["Counter_Value"])
best = {}
for (n, g, d), v in per.items():  # keep the largest launch per kernel name (the 131,072-row one)
    if n not in best or v.get("GRBM_GUI_ACTIVE", 0) > best[n].get("GRBM_GUI_ACTIVE", 0):
        best[n] = dict(v)
kt = {}  # kernel durations (ns) from the trace of the same run, by dispatch
for r in csv.DictReader(open(glob.glob("gpurun_out/f1tsq/sq/**/*kernel_trace.csv", recursive=True)[0])):
    kt[r["Kernel_Name"][:72]] = max(kt.get(r["Kernel_Name"][:72], 0), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for n, v in best.items():
    wc = v.get("SQ_WAVE_CYCLES", 0) or 1
    # 1,024 SIMDs; GRBM_GUI_ACTIVE sums the 8 XCDs' cycles
    v["mfma_util"] = v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (1024 * v.get("GRBM_GUI_ACTIVE", 1) / 8)
    if kt.get(n):
        v["duration_ms"] = kt[n] / 1e6
        v["clock_ghz"] = v.get("GRBM_GUI_ACTIVE", 0) / 8 / kt[n]
    v["mfma_busy_per_busy_cycle"] = v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(v.get("SQ_BUSY_CYCLES", 1), 1)
    v["wait_any_share"] = v.get("SQ_WAIT_ANY", 0) / wc
    v["wait_inst_any_share"] = v.get("SQ_WAIT_INST_ANY", 0) / wc
    v["active_inst_share"] = v.get("SQ_ACTIVE_INST_ANY", 0) / wc
print(json.dumps(best, indent=1))
json.dump(best, open("gpurun_out/f1tsq/summary.json", "w"), indent=1)
PY
find $O -name "*.csv" -size +5M -delete
