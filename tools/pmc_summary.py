"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over tools/kernel_bench.py --only logprob
into per-launch HBM traffic for the log-prob kernels (profiles/<round>/pmc_logprob.json).

Corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are KiB; on gfx950 FETCH_SIZE
reports half the bytes of a wide coalesced streaming read -> x2; WRITE_SIZE is exact for 16-B
streaming stores.

  python tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write ROWS VOCAB OUT.json
"""

import csv
import glob
import json
import statistics
import sys


def load(d, counter):
    path = glob.glob(f"{d}/*counter_collection.csv")[0]
    out = {}
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"]
        if "logprob_entropy" not in n or r["Counter_Name"] != counter:
            continue
        k = "logprob_entropy_fwd" if "fwd" in n else "logprob_entropy_bwd"
        out.setdefault(k, []).append(float(r["Counter_Value"]))
    return {k: statistics.median(v) for k, v in out.items()}


def main():
    fetch_dir, write_dir, rows, vocab, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    f = load(fetch_dir, "FETCH_SIZE")
    w = load(write_dir, "WRITE_SIZE")
    algo = {"logprob_entropy_fwd": rows * (2 * vocab + 20), "logprob_entropy_bwd": rows * (4 * vocab + 28)}
    res = {"rows_per_launch": rows, "vocab": vocab, "dtype": "bf16", "kernels": {}}
    for k in algo:
        fetch_b = f[k] * 1024 * 2
        write_b = w[k] * 1024
        tot = fetch_b + write_b
        res["kernels"][k] = {
            "fetch_size_kib_raw": f[k], "write_size_kib_raw": w[k],
            "fetch_bytes_corrected": fetch_b, "write_bytes": write_b, "traffic_bytes": tot,
            "traffic_bytes_per_row": tot / rows, "algo_bytes": algo[k], "traffic_over_algo": tot / algo[k],
        }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
