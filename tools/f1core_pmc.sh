#!/bin/bash
# PMC passes over the f1 core bench (variant $1): LDS bank conflicts / MFMA busy, then L2 hit rate
set -u
O=gpurun_out/f1pmc
mkdir -p $O
export TMPDIR=/tmp
V=${1:-3}
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/lds -o run -- python3 tools/f1core_bench.py --variants $V --iters 2 > $O/lds.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/tcc -o run -- python3 tools/f1core_bench.py --variants $V --iters 2 > $O/tcc.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob, collections
for d in ("lds", "tcc"):
    p = glob.glob(f"gpurun_out/f1pmc/{d}/**/*counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.Counter()
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"][:60]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[(k, r["Counter_Name"])] += 1
    for k, v in agg.items():
        if "gemm_nt" in k or "Cijk" in k:
            print(d, k, {c: round(x / max(1, cnt[(k, c)]), 1) for c, x in v.items()})
PY
find $O -name "*.csv" -size +5M -delete
