# round 4 GPU pass m: flash attention on the bench's packed micro-batch: times, then SQ counters
# (MFMA busy, clock, waits, VALU share) of the forward and the two backward kernels
set -o pipefail
O=gpurun_out/r04/attn_sq
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 python tools/attn_ab.py --tag base > $O/time.jsonl 2> $O/time.err || { tail $O/time.err; exit 1; }
cat $O/time.jsonl
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
timeout -s KILL 200 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/sq -o run -- python3 tools/attn_ab.py --tag sq > $O/sq.log 2>&1 || { echo "sq FAILED"; tail $O/sq.log; exit 1; }
python3 tools/sq_summary.py $O/sq flash_fwd flash_bwd_dq flash_bwd_dkdv | tee $O/sq.jsonl
