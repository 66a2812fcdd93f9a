#!/bin/bash
# PMC passes over the f1 v3 kernel (tools/f1core/f1t.hip) at 131,072 x 896 x 151,936, 8 vocab ranges:
# beyond-L2 traffic (FETCH_SIZE, x2 on gfx950) and the L2 hit rate, with (variant 1) and without
# (variant 2) the XCD remap of the (row block, range) grid, next to hipBLASLt's lm_head GEMM.
set -u
O=gpurun_out/f1tpmc
mkdir -p $O
export TMPDIR=/tmp
for pass in fetch tcc; do
  if [ $pass = fetch ]; then C="FETCH_SIZE"; else C="TCC_HIT_sum TCC_MISS_sum"; fi
  timeout -s KILL 180 rocprofv3 --pmc $C --output-format csv -d $O/$pass -o run -- python3 tools/f1t_bench.py --rows 131072 --splits 8 --variants 1 2 --iters 1 --no-product > $O/$pass.log 2>&1 || exit $?
done
python3 - <<'PY'
import csv, glob, collections, json
res = {}
for d in ("fetch", "tcc"):
    p = glob.glob(f"gpurun_out/f1tpmc/{d}/**/*counter_collection.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(p)))
    per = collections.defaultdict(list)
    for r in rows:
        n = r["Kernel_Name"]
        if "lp_t_kernel" in n or "Cijk" in n:
            remap = ("true>" in n) or ("Lb1E" in n)
            key = ("lp_t_kernel<1,true> (remap)" if remap else "lp_t_kernel<1,false> (no remap)") if "lp_t" in n else n[:40]
            per[(key, r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in per.items():
        big = [x for x in v]
        res.setdefault(k, {})[c] = max(big)  # the 131,072-row launches are the largest
for k, v in res.items():
    if "FETCH_SIZE" in v:
        v["fetch_bytes_x2"] = v["FETCH_SIZE"] * 1024 * 2
    if "TCC_HIT_sum" in v:
        v["l2_hit_rate"] = v["TCC_HIT_sum"] / (v["TCC_HIT_sum"] + v["TCC_MISS_sum"])
print(json.dumps(res, indent=1))
json.dump(res, open("gpurun_out/f1tpmc/summary.json", "w"), indent=1)
PY
find $O -name "*.csv" -size +5M -delete
