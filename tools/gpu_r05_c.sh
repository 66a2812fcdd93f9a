# round 5 GPU pass c: (1) the f1 in-step penalty: f1 standalone, f1 right after
# back-to-back GEMM load, and SQ/GRBM counters (MFMA busy, clock) of f1 in the bench step vs
# standalone; (2) the interleaved A/B of the step boundary (VERL_AMD_BLOCKING_STEP_BOUNDARY=1 = the
# round-4 blocking metric readback + mask copy) on the full batch and the 8-prompt per-rank workload
set -o pipefail
O=gpurun_out/r05/c
mkdir -p $O
for pre in 0 400; do
  for it in 1 4; do
    timeout -k 10 200 python tools/f1_ab.py --iters $it --pre-gemm-ms $pre >> $O/f1_pre_gemm.jsonl 2>> $O/f1_pre_gemm.err || { echo "f1_ab FAILED"; tail $O/f1_pre_gemm.err; exit 1; }
  done
done
cat $O/f1_pre_gemm.jsonl | cut -c1-200
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE"
timeout -s KILL 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/sq_step -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-kernel-timing --out $O/sq_step_bench.json > $O/sq_step.log 2>&1 || { echo "sq step FAILED"; tail $O/sq_step.log; exit 1; }
echo "== in step"; python3 tools/sq_summary.py $O/sq_step linear_logprob_t256 Custom_Cijk_Alik_Bljk_BBS_BH_Bias_HA_S_SAV_NTD_SK3 logprob_entropy_fwd | tee $O/sq_step.jsonl
timeout -s KILL 200 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/sq_alone -o run -- python3 tools/f1_ab.py --iters 2 --unfused > $O/sq_alone.log 2>&1 || { echo "sq alone FAILED"; tail $O/sq_alone.log; exit 1; }
echo "== standalone"; python3 tools/sq_summary.py $O/sq_alone linear_logprob_t256 Cijk logprob_entropy_fwd | tee $O/sq_alone.jsonl
find $O -name "*counter_collection.csv" -size +20M -delete
bash tools/gpu_ab.sh step_boundary 2 "VERL_AMD_BLOCKING_STEP_BOUNDARY=1 --prompts 8" "--prompts 8" "VERL_AMD_BLOCKING_STEP_BOUNDARY=1" "" > $O/step_boundary_ab.txt 2>&1 || { echo "AB FAILED"; cat $O/step_boundary_ab.txt; exit 1; }
cat $O/step_boundary_ab.txt
