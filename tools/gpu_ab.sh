#!/bin/bash
# Interleaved same-box A/B of bench.py (or any command) variants: the one driver behind every
# A/B recorded under profiles/ (allocator segments, HIP env, clip, dgrad layout, log-prob
# micro-batch, attention library swap, warm-up sensitivity, ...).
#
# usage: tools/gpu_ab.sh NAME REPEATS VARIANT [VARIANT ...] [-- COMMON_BENCH_ARGS...]
#   VARIANT  whitespace-separated tokens: VAR=VALUE sets an environment variable for that run,
#            --flag / value tokens are extra bench.py arguments, e.g.
#              "HIP_FORCE_DEV_KERNARG=1"  "HIP_FORCE_DEV_KERNARG=0 --prompts 8"
#   AB_CMD   (env) command run instead of "python bench.py" (its stdout's JSON line is kept)
# Runs REPEATS rounds of all variants in order, one process each, under its own time limit;
# stops at the first failing run. Prints one line per run: variant, value, ms/step, peak HBM.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
NAME=$1; REPS=$2; shift 2
VARIANTS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do VARIANTS+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
COMMON=("$@")
O=gpurun_out/ab_$NAME
mkdir -p "$O"
CMD=${AB_CMD:-"python bench.py --no-cpu-baseline --steps 3 --warmup 1"}
i=0
for r in $(seq 1 "$REPS"); do
  for v in "${VARIANTS[@]}"; do
    i=$((i + 1))
    envs=(); args=()
    for tok in $v; do
      if [[ $tok =~ ^[A-Z_][A-Z0-9_]*= ]]; then envs+=("$tok"); else args+=("$tok"); fi
    done
    env "${envs[@]}" timeout -k 10 400 $CMD "${COMMON[@]}" "${args[@]}" > "$O/run_$i.json" 2> "$O/run_$i.err" || exit $?
    python3 - "$O/run_$i.json" "$v" <<'PY'
import json, sys
recs = [json.loads(x) for x in open(sys.argv[1]) if x.startswith("{")]
d = recs[-1] if recs else {}
cfg = d.get("config", {})
print(f"{sys.argv[2]!r:50s}", d.get("value"), d.get("ms_per_step"), cfg.get("peak_hbm_gb"), flush=True)
PY
  done
done
