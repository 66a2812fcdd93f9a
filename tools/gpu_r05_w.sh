# round 5 GPU pass w: the f1 sweep without per-step 64-bit divisions (incremental step counters)
# and with the wave-row skew (VA_TUNE_F1_SKEW = 21), interleaved against the previous build
# (verl_amd/lib/ab/libverl_amd_div.so) at the bench shape (131,072 x 896 x 151,936); then the
# linear_logprob / gate_up_swiglu parity tests on the new build
set -o pipefail
O=gpurun_out/r05/w
mkdir -p $O
OLD=verl_amd/lib/ab/libverl_amd_div.so
for i in 1 2 3; do
  VERL_AMD_LIB=$OLD timeout -k 10 120 python tools/f1_ab.py --tag div_skew0 >> $O/f1_counter_ab.jsonl 2>> $O/f1_ab.err || { echo "old FAILED"; tail -20 $O/f1_ab.err; exit 1; }
  for sk in 0 1; do
    timeout -k 10 120 python tools/f1_ab.py --tag counters_skew$sk --tune 21=$sk >> $O/f1_counter_ab.jsonl 2>> $O/f1_ab.err || { echo "skew $sk FAILED"; tail -20 $O/f1_ab.err; exit 1; }
  done
done
cat $O/f1_counter_ab.jsonl
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_linear_logprob_gpu.py tests/test_model_ops_gpu.py -k "linear or logprob or gate_up or fused" > $O/pytest_f1.log 2>&1 || { echo "TESTS FAILED"; tail -30 $O/pytest_f1.log; exit 1; }
tail -3 $O/pytest_f1.log
