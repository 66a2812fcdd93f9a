#!/bin/bash
# One parameterised GPU pass (round 6 on; replaces the per-pass tools/gpu_r0*.sh records): every
# step runs under its own time limit, steps are chained (the pass stops at the first failure), and
# each output file starts with the exact command that produced it ("# cmd: ..." for text / JSONL;
# a .cmd sidecar for JSON). COMMANDS.txt in the output directory lists every step, its exit status
# and wall time.
#
# usage: tools/gpu_pass.sh OUTDIR STEP [STEP ...]
#   suite                 full GPU test suite              -> pytest_gpu.log
#   tests:<pytest args>   a subset, e.g. "tests:tests/test_weight_grad_gpu.py -k tile" -> pytest_<n>.log
#   smoke                 __graft_entry__.smoke()          -> smoke.log
#   bench[:<tag>[:<args>]] bench.py as the driver runs it (+ args) -> bench_<tag>.json / .log
#   rocprof[:<tag>[:<args>]] the bench command (+ args) under rocprofv3 --kernel-trace --stats -> kernel_stats_<tag>*,
#                         trace_gaps_<tag>.txt, bench_under_rocprof_<tag>.json
#   pmc_f1                tools/f1_pmc.sh                  -> pmc_f1_product.json
#   tool:<script> <args>  python tools/<script> <args>     -> <script stem>[_<n>].jsonl
#   ab:<name>:<reps>:<v1>|<v2>[|...][:<common args>]   tools/gpu_ab.sh (interleaved bench variants) -> ab_<name>.txt
#   sq:<name>:<kernel substrings>:<command>   one rocprofv3 --pmc pass of the SQ / GRBM counters over
#                         <command> (no other trace domains), summarised by tools/sq_summary.py -> sq_<name>.jsonl
#   pmc:<name>:<counters, comma-separated>:<kernel substrings>:<command>   the same with other counters
#                         (at most 8 SQ_ per pass) -> sq_<name>.jsonl ("extra": per-dispatch averages)
#   cmd:<name>:<command>  any other command                -> <name>.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=$1; shift
mkdir -p "$O"
export TMPDIR=/tmp
export VA_REHEARSAL_OUT=$O/rehearsal
n=0
log_cmd() { echo "$(date -u +%H:%M:%S) rc=$2 ${3}s :: $1" >> "$O/COMMANDS.txt"; }
run() {  # run LIMIT OUTFILE CMD...: stdout to OUTFILE (headed by the command), stderr to OUTFILE.err
  local lim=$1 out=$2; shift 2
  local t0=$SECONDS
  { echo "# cmd: $*"; } > "$out"
  timeout -k 10 "$lim" "$@" >> "$out" 2> "$out.err"
  local rc=$?
  log_cmd "$*" $rc $((SECONDS - t0))
  if [ $rc -ne 0 ]; then echo "STEP FAILED rc=$rc: $*"; tail -30 "$out"; tail -30 "$out.err"; exit $rc; fi
}
for step in "$@"; do
  n=$((n + 1))
  case "$step" in
    suite)
      run 1100 "$O/pytest_gpu.log" python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread
      tail -1 "$O/pytest_gpu.log" ;;
    tests:*)
      # shellcheck disable=SC2086
      run 900 "$O/pytest_$n.log" python -u -m pytest ${step#tests:} -x -v --timeout 300 --timeout-method thread
      tail -1 "$O/pytest_$n.log" ;;
    smoke)
      run 300 "$O/smoke.log" python -c "import __graft_entry__ as g; g.smoke()"
      tail -1 "$O/smoke.log" ;;
    bench*)
      IFS=: read -r _ tag args <<< "$step"; tag=${tag:-default}
      # shellcheck disable=SC2086
      run 500 "$O/bench_$tag.log" python bench.py --out "$O/bench_$tag.json" $args
      echo "# cmd: python bench.py --out $O/bench_$tag.json $args" > "$O/bench_$tag.json.cmd"
      python -c "import json;d=json.load(open('$O/bench_$tag.json'));r=d['roofline'];print('bench $tag', d['value'], d['ms_per_step'], r['kernel'], r['frac'], d.get('config',{}).get('peak_hbm_gb'))" ;;
    rocprof*)
      IFS=: read -r _ tag args <<< "$step"; tag=${tag:-headline}
      # shellcheck disable=SC2086
      run 600 "$O/bench_prof_$tag.log" rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$tag" -o "$tag" -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --out "$O/bench_under_rocprof_$tag.json" $args
      st=$(find "$O/prof_$tag" -name "*kernel_stats.csv" | head -1)
      kt=$(find "$O/prof_$tag" -name "*kernel_trace.csv" | head -1)
      { echo "# cmd: rocprofv3 --kernel-trace --stats -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline; python tools/prof_summary.py"; python tools/prof_summary.py "$st"; } > "$O/kernel_stats_${tag}_summary.txt"
      cp "$st" "$O/kernel_stats_$tag.csv"
      { echo "# cmd: python tools/trace_gaps.py <kernel_trace> --steps 3 --top 12"; python tools/trace_gaps.py "$kt" --steps 3 --top 12 | tail -16; } > "$O/trace_gaps_$tag.txt"
      gzip -c "$kt" > "$O/kernel_trace_$tag.csv.gz" && rm -rf "$O/prof_$tag"
      head -14 "$O/kernel_stats_${tag}_summary.txt" ;;
    pmc_f1)
      run 600 "$O/f1_pmc.log" bash tools/f1_pmc.sh
      cp gpurun_out/f1pmc/summary.json "$O/pmc_f1_product.json"
      echo "# cmd: bash tools/f1_pmc.sh" > "$O/pmc_f1_product.json.cmd" ;;
    tool:*)
      t=${step#tool:}; script=${t%% *}; stem=$(basename "$script" .py)
      [ "$t" = "$script" ] && targs="" || targs=${t#* }
      # shellcheck disable=SC2086
      run 900 "$O/${stem}_$n.jsonl" python "tools/$script" $targs
      tail -8 "$O/${stem}_$n.jsonl" ;;
    ab:*)
      IFS=: read -r _ name reps vars common <<< "$step"
      IFS='|' read -r -a varr <<< "$vars"
      # shellcheck disable=SC2086
      run 1100 "$O/ab_$name.txt" bash tools/gpu_ab.sh "$name" "$reps" "${varr[@]}" -- $common
      cat "$O/ab_$name.txt" ;;
    sq:*)
      IFS=: read -r _ name subs cmd <<< "$step"
      C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE"
      # shellcheck disable=SC2086
      run 200 "$O/sq_$name.log" timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$O/sq_$name" -o run -- $cmd
      # shellcheck disable=SC2086
      { echo "# cmd: rocprofv3 --pmc $C --kernel-trace -- $cmd; python tools/sq_summary.py <dir> $subs"; python tools/sq_summary.py "$O/sq_$name" $subs; } > "$O/sq_$name.jsonl"
      rm -rf "$O/sq_$name"
      cat "$O/sq_$name.jsonl" ;;
    pmc:*)
      IFS=: read -r _ name cnt subs cmd <<< "$step"
      C=${cnt//,/ }
      # shellcheck disable=SC2086
      run 200 "$O/sq_$name.log" timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$O/sq_$name" -o run -- $cmd
      # shellcheck disable=SC2086
      { echo "# cmd: rocprofv3 --pmc $C --kernel-trace -- $cmd; python tools/sq_summary.py <dir> $subs"; python tools/sq_summary.py "$O/sq_$name" $subs; } > "$O/sq_$name.jsonl"
      rm -rf "$O/sq_$name"
      cat "$O/sq_$name.jsonl" ;;
    cmd:*)
      IFS=: read -r _ name cmd <<< "$step"
      # shellcheck disable=SC2086
      run 900 "$O/$name.txt" $cmd
      tail -12 "$O/$name.txt" ;;
    *) echo "unknown step: $step"; exit 2 ;;
  esac
done
