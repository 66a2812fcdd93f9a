"""Per-(kernel, grid) device times from a rocprofv3 --kernel-trace CSV.

rocprofv3's --stats summary averages a kernel over all its launches; a microbenchmark that runs
the same kernel at several batch sizes needs the durations split by launch shape. Prints one
JSON record per (kernel, grid) with the launch count and the mean / median duration in us, and,
when --bytes KERNEL_SUBSTR=BYTES_PER_TOKEN:TOKENS_PER_GRID_ITEM is given, the achieved GB/s.

Usage: python tools/prof_split.py run_kernel_trace.csv [--match verl_amd_substr ...]
"""

from __future__ import annotations

import argparse
import re
import csv
import json
import statistics
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--match", nargs="*", default=[])
    ap.add_argument("--min-launches", type=int, default=1)
    ap.add_argument("--phases", type=int, default=1,
                    help="split each (kernel, grid) series, in launch order, into this many equal parts "
                         "(kernels whose grid does not change with the batch size)")
    args = ap.parse_args()
    groups = defaultdict(list)
    with open(args.trace) as f:
        for row in sorted(csv.DictReader(f), key=lambda r: int(r["Start_Timestamp"])):
            name = row["Kernel_Name"]
            if args.match and not any(m in name for m in args.match):
                continue
            grid = (int(row["Grid_Size_X"]), int(row["Grid_Size_Y"]), int(row["Grid_Size_Z"]))
            dur = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3
            m = re.search(r"(\w+_kernel(?:<[^>]*>)?)", name)
            short = m.group(1) if m else name.split("(")[0].replace("void ", "")
            groups[(short, grid)].append(dur)
    for (name, grid), d in sorted(groups.items()):
        if len(d) < args.min_launches:
            continue
        n = args.phases if len(d) % args.phases == 0 else 1
        k = len(d) // n
        for ph in range(n):
            x = d[ph * k : (ph + 1) * k]
            rec = {"kernel": name, "grid": grid, "launches": len(x), "mean_us": round(statistics.mean(x), 3),
                   "median_us": round(statistics.median(x), 3), "min_us": round(min(x), 3)}
            if n > 1:
                rec["phase"] = ph
            print(json.dumps(rec))


if __name__ == "__main__":
    main()
