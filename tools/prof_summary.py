"""Summarise a rocprofv3 *_kernel_stats.csv by kernel family (GEMM, attention, elementwise, ours)."""
import csv
import re
import sys


def family(name: str) -> str:
    if name.startswith("Cijk") or name.startswith("Custom_Cijk"):
        return "gemm (hipBLASLt)"
    if "attn" in name or name.startswith("bwd_kernel"):
        return "attention (flash varlen)"
    if "va::" in name or "logprob_entropy" in name or "ppo_loss" in name or "gae_scan" in name or "outcome_adv" in name:
        return "verl_amd HIP kernels"
    if "copy" in name.lower() or "Cat" in name:
        return "copies / casts"
    if "elementwise" in name or "Functor" in name or "reduce" in name.lower():
        return "torch elementwise / reductions"
    return "other"


def main(path):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    fam = {}
    for r in rows:
        f = family(r["Name"])
        fam.setdefault(f, [0.0, 0])
        fam[f][0] += float(r["TotalDurationNs"])
        fam[f][1] += int(r["Calls"])
    print(f"total kernel time {tot / 1e6:.1f} ms")
    for f, (t, c) in sorted(fam.items(), key=lambda kv: -kv[1][0]):
        print(f"  {f:34s} {t / 1e6:9.1f} ms  {100 * t / tot:5.1f}%  {c:7d} launches")
    print("top 25 kernels:")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
        print(f"  {r['Name'][:70]:70s} {float(r['TotalDurationNs']) / 1e6:8.1f} ms calls {r['Calls']:>6s} avg {float(r['AverageNs']) / 1e3:8.1f} us")
    print("ours:")
    for r in rows:
        if family(r["Name"]) == "verl_amd HIP kernels":
            n = re.sub(r"^void ", "", r["Name"]).replace("(anonymous namespace)::", "")
            n = re.sub(r"\(.*", "", n) or n
            n = n[:90]
            print(f"  {n:90s} calls {r['Calls']:>6s} avg {float(r['AverageNs']) / 1e3:9.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
