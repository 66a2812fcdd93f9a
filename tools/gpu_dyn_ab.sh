#!/bin/bash
# use_dynamic_bsz A/B on the realistic (U[128, 1024]) variant at the reference's 16,384-token budget:
# reference passes | larger no-grad log-prob passes | merged update passes | both; two rounds, interleaved
set -u
mkdir -p gpurun_out
out=gpurun_out/dyn_ab.jsonl
: > $out
for round in 1 2; do
  for cfg in "0 0" "151552 0" "0 151552" "151552 151552"; do
    set -- $cfg
    timeout -k 10 300 python bench.py --steps 3 --warmup 1 --responses realistic --dynamic-bsz 16384 \
      --logprob-max-tokens $1 --compute-max-tokens $2 > gpurun_out/dyn_ab_cur.json 2> gpurun_out/dyn_ab_cur.err || exit $?
    python - "$round" "$1" "$2" >> $out <<'PY'
import json, sys
d = json.loads(open("gpurun_out/dyn_ab_cur.json").read().strip().splitlines()[-1])
c = d["config"]
print(json.dumps({"round": int(sys.argv[1]), "logprob_max_tokens": int(sys.argv[2]), "compute_max_tokens": int(sys.argv[3]),
                  "tokens_per_s": d["value"], "ms_per_step": d["ms_per_step"], "peak_hbm_gb": c["peak_hbm_gb"]}))
PY
    tail -1 $out
  done
done
