"""HBM traffic per (kernel, grid) from rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE passes (separate
runs of the same command), with the gfx950 corrections of MI355X_MICROARCH.md §HBM: both counters
are KiB; FETCH_SIZE reports half the bytes of wide coalesced streaming reads (x2); WRITE_SIZE is
exact for 16-byte streaming stores.

  python tools/pmc_split.py FETCH_DIR WRITE_DIR [--match substr ...]
prints one JSON record per (kernel, grid): median corrected fetch / write bytes per launch.
"""

from __future__ import annotations

import argparse
import csv
import glob
import json
import re
import statistics
from collections import defaultdict


def load(d, counter, match):
    path = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    out = defaultdict(list)
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"]
        if r["Counter_Name"] != counter or (match and not any(m in n for m in match)):
            continue
        m = re.search(r"(\w+_kernel(?:<[^>]*>)?)", n)
        k = m.group(1) if m else n.split("(")[0]
        grid = r.get("Grid_Size") or r.get("Grid_Size_X") or "?"
        out[(k, grid)].append(float(r["Counter_Value"]))
    return {k: statistics.median(v) for k, v in out.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--match", nargs="*", default=[])
    args = ap.parse_args()
    f = load(args.fetch_dir, "FETCH_SIZE", args.match)
    w = load(args.write_dir, "WRITE_SIZE", args.match)
    for key in sorted(set(f) | set(w)):
        fb = f.get(key, 0.0) * 1024 * 2
        wb = w.get(key, 0.0) * 1024
        print(json.dumps({"kernel": key[0], "grid": key[1], "fetch_bytes_corrected": fb, "write_bytes": wb,
                          "traffic_bytes": fb + wb}))


if __name__ == "__main__":
    main()
