# round 5 GPU pass x: the f1 sweep with per-lane staging offsets computed once (scalar tile / chunk
# base per K-step) vs the step-counter build (verl_amd/lib/ab/libverl_amd_counters.so), interleaved
# at the bench shape; the fused backward's dlogits kernel likewise; then the parity tests
set -o pipefail
O=gpurun_out/r05/x
mkdir -p $O
OLD=verl_amd/lib/ab/libverl_amd_counters.so
for i in 1 2 3; do
  VERL_AMD_LIB=$OLD timeout -k 10 120 python tools/f1_ab.py --tag counters >> $O/f1_offsets_ab.jsonl 2>> $O/f1_ab.err || { echo "old FAILED"; tail -20 $O/f1_ab.err; exit 1; }
  timeout -k 10 120 python tools/f1_ab.py --tag offsets >> $O/f1_offsets_ab.jsonl 2>> $O/f1_ab.err || { echo "new FAILED"; tail -20 $O/f1_ab.err; exit 1; }
done
cat $O/f1_offsets_ab.jsonl
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_linear_logprob_gpu.py tests/test_model_ops_gpu.py tests/test_reference_protocol_gpu.py tests/test_fused_backends_gpu.py > $O/pytest_f1.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/pytest_f1.log; exit 1; }
tail -3 $O/pytest_f1.log
