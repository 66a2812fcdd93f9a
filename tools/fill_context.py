"""Where the small zero-fill kernels of a step come from: each FillFunctor launch in a rocprofv3
kernel trace counted by its nearest preceding / following non-fill kernel (tools/gpu_fill_context.sh)."""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"].replace("(anonymous namespace)::", "") for r in rows]


def short(n):
    n = n.replace("void ", "")
    return n.split("(")[0][-56:] if not n.startswith("Cijk") and not n.startswith("Custom") else "GEMM"


def is_fill(n):
    return "FillFunctor" in n


def near(i, step):
    j = i + step
    while 0 <= j < len(rows) and is_fill(names[j]):
        j += step
    return short(names[j]) if 0 <= j < len(rows) else "-"


agg = collections.defaultdict(lambda: [0, 0.0])
for i, r in enumerate(rows):
    if is_fill(names[i]):
        key = (near(i, -1), near(i, 1), int(r["Grid_Size_X"]))
        agg[key][0] += 1
        agg[key][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
tot = sum(v[0] for v in agg.values())
print(f"{tot} fills, {sum(v[1] for v in agg.values()) / 1e3:.2f} ms")
for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:25]:
    print(f"{n:5d}x {t / 1e3:7.2f} ms  grid={k[2]:<9} {k[0]} -> {k[1]}")
