# round 5 GPU pass ao: SQ / GRBM counters of f1 after the staging rework (MFMA busy, clock, wait
# share) standalone next to the unfused hipBLASLt lm_head GEMM, then the full GPU suite + smoke()
set -o pipefail
O=gpurun_out/r05/ao
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE"
timeout -s KILL 200 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/sq_alone -o run -- python3 tools/f1_ab.py --iters 2 --unfused > $O/sq_alone.log 2>&1 || { echo "sq alone FAILED"; tail $O/sq_alone.log; exit 1; }
python3 tools/sq_summary.py $O/sq_alone linear_logprob_t256 Cijk logprob_entropy_fwd | tee $O/sq_alone.jsonl
find $O -name "*counter_collection.csv" -size +20M -delete
export VA_REHEARSAL_OUT=$O/rehearsal
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest FAILED"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke FAILED"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
