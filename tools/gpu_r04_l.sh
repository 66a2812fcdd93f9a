# round 4 GPU pass l: backbone weight gradients at the bench's update micro-batch, own kernel vs
# hipBLASLt: times, then SQ counters per shape (MFMA busy, clock, waits)
set -o pipefail
O=gpurun_out/r04/wgrad_sq
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python tools/wgrad_sq.py > $O/time.jsonl 2> $O/time.err || { tail $O/time.err; exit 1; }
cat $O/time.jsonl
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE"
for s in gateup down qkv o; do
  timeout -s KILL 150 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/sq_$s -o run -- python3 tools/wgrad_sq.py --shape $s --iters 1 > $O/sq_$s.log 2>&1 || { echo "sq $s FAILED"; tail $O/sq_$s.log; exit 1; }
  echo "== $s"; python3 tools/sq_summary.py $O/sq_$s wgrad_kernel wgrad_reduce Cijk | tee $O/sq_$s.jsonl
done
