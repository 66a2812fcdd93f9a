"""Per-kernel MFMA busy share, clock and wait share from one rocprofv3 --pmc run (csv output) with
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY
SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE (or SQ_ACTIVE_INST_VALU: VALU share of wave time). For every kernel-name substring given, the
dispatches whose name holds it are averaged (MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES over 1,024 SIMDs x
GRBM_GUI_ACTIVE / 8 XCDs; clock = GRBM_GUI_ACTIVE / 8 / traced duration).

  python tools/sq_summary.py <rocprof dir> <substring> [<substring> ...]
"""

import collections
import csv
import glob
import json
import sys


FIXED = {"SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
         "SQ_ACTIVE_INST_ANY", "SQ_INSTS_VALU", "GRBM_GUI_ACTIVE", "SQ_ACTIVE_INST_VALU"}


def main():
    d, names = sys.argv[1], sys.argv[2:]
    cc = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    kt = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    kname = {}
    for r in csv.DictReader(open(cc)):
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        kname[r["Dispatch_Id"]] = r["Kernel_Name"]
    dur = {}
    for r in csv.DictReader(open(kt)):
        dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for sub in names:
        ids = [i for i in per if sub in kname[i] and dur.get(i)]
        if not ids:
            print(json.dumps({"kernel": sub, "dispatches": 0}))
            continue
        busy = clock = wait = us = valu = 0.0
        extra = collections.defaultdict(float)
        for i in ids:
            v = per[i]
            g = v.get("GRBM_GUI_ACTIVE", 0.0) / 8
            busy += v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (1024 * g) if g else 0.0
            clock += g / dur[i]
            wait += v.get("SQ_WAIT_ANY", 0.0) / (v.get("SQ_WAVE_CYCLES") or 1)
            valu += v.get("SQ_ACTIVE_INST_VALU", 0.0) / (v.get("SQ_WAVE_CYCLES") or 1)
            us += dur[i] / 1e3
            for c, x in v.items():
                if c not in FIXED:
                    extra[c] += x
        n = len(ids)
        print(json.dumps({"kernel": sub, "dispatches": n, "avg_us": round(us / n, 1),
                          "mfma_busy": round(busy / n, 3), "clock_ghz": round(clock / n, 3),
                          "busy_x_clock": round(busy * clock / n / n, 3), "wait_share": round(wait / n, 3),
                          "valu_active_share": round(valu / n, 3),
                          "extra": {c: round(x / n) for c, x in extra.items()}, "name": kname[ids[0]][:90]}))


if __name__ == "__main__":
    main()
