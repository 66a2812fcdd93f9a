"""Per-step kernel shares from a rocprofv3 kernel trace (csv or csv.gz): the steps are cut at the
optimizer launches (va_adamw_flat, or torch's multi-tensor AdamW), and for each of the last N steps
this prints the launch count, span, kernel time and the share of torch / rocPRIM kernels (fills,
reductions, elementwise, copies) — the fixed per-step device work VERDICT r5 #3 asks about.

  python tools/step_kernel_share.py <kernel_trace.csv[.gz]> [--steps 3]
"""

import argparse
import csv
import gzip


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    op = gzip.open if args.trace.endswith(".gz") else open
    rows = sorted(csv.DictReader(op(args.trace, "rt")), key=lambda r: int(r["Start_Timestamp"]))
    opt = [i for i, r in enumerate(rows) if "adamw_flat_kernel" in r["Kernel_Name"]
           or ("multi_tensor_apply_kernel" in r["Kernel_Name"] and "Adam" in r["Kernel_Name"])]
    groups = []
    for i in opt:
        if groups and i - groups[-1][-1] <= 3:
            groups[-1].append(i)
        else:
            groups.append([i])

    def dur(r):
        return int(r["End_Timestamp"]) - int(r["Start_Timestamp"])

    tot_all = tor_all = 0
    for gi in range(max(1, len(groups) - args.steps), len(groups)):
        seg = rows[groups[gi - 1][-1] + 1 : groups[gi][-1] + 1]
        tot = sum(dur(r) for r in seg)
        small = [r for r in seg if "at::native" in r["Kernel_Name"] or "rocprim" in r["Kernel_Name"]
                 or "__amd_rocclr" in r["Kernel_Name"]]
        tor = sum(dur(r) for r in small)
        span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e6
        print(f"step {gi}: {len(seg)} launches, span {span:.1f} ms, kernel time {tot / 1e6:.1f} ms, "
              f"torch / rocPRIM / copies {tor / 1e6:.2f} ms in {len(small)} launches = {100 * tor / tot:.2f} %")
        tot_all += tot
        tor_all += tor
    print(f"last {args.steps} steps: torch / rocPRIM / copies share {100 * tor_all / max(tot_all, 1):.2f} %")


if __name__ == "__main__":
    main()
