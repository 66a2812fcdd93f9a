"""Which op each hipBLASLt GEMM launch belongs to, from a rocprofv3 kernel trace: GEMM kernels are
grouped by (kernel tail, workgroups) and labelled with the nearest preceding and following
non-GEMM kernel (tools/gpu_gemm_context.sh)."""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
names = [r["Kernel_Name"].replace("(anonymous namespace)::", "") for r in rows]


def short(n):
    return n.split("(")[0].replace("void ", "")[-48:]


def is_gemm(n):
    return n.startswith("Custom_Cijk") or n.startswith("Cijk")


def near(i, step):
    j = i + step
    while 0 <= j < len(rows) and is_gemm(names[j]):
        j += step
    return short(names[j]) if 0 <= j < len(rows) else "-"


agg = collections.defaultdict(lambda: [0.0, 0])
for i, r in enumerate(rows):
    if not is_gemm(names[i]):
        continue
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    wgs = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
    key = (names[i].split("_MT")[-1][:14] if "_MT" in names[i] else names[i][-30:], "SK" in names[i], wgs,
           near(i, -1), near(i, 1))
    agg[key][0] += dur
    agg[key][1] += 1
for k, (t, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:28]:
    print(f"{t / 1e3:8.1f} ms {n:4d}x avg {t / n:8.1f} us  MT{k[0]:<14} sk={int(k[1])} wgs={k[2]:<6} {k[3]} -> {k[4]}")
