# NOTE: records the run at commit fdf044b (the VA_F1_SCHED code was removed after it).
# round 4 GPU pass k: f1 fragment-read pipelining (VA_F1_SCHED build: asm ds_read one MFMA group
# ahead + counted lgkmcnt) vs the product build; forward and fused backward, alternated; the
# linear-logprob parity tests on the variant build
set -o pipefail
O=gpurun_out/r04/sched
mkdir -p $O
V=verl_amd/lib/ab/libverl_amd_sched.so
for r in 1 2; do
  timeout -k 10 120 python tools/f1_ab.py --tag base >> $O/f1_fwd.jsonl || exit 1
  VERL_AMD_LIB=$V timeout -k 10 120 python tools/f1_ab.py --tag sched >> $O/f1_fwd.jsonl || exit 1
done
cat $O/f1_fwd.jsonl
timeout -k 10 200 python tools/f1_bwd_ab.py > $O/f1_bwd_base.json && VERL_AMD_LIB=$V timeout -k 10 200 python tools/f1_bwd_ab.py > $O/f1_bwd_sched.json || exit 1
cat $O/f1_bwd_base.json $O/f1_bwd_sched.json
VERL_AMD_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_linear_logprob_gpu.py -m gpu -x -q --timeout 250 --timeout-method thread > $O/pytest_sched.log 2>&1; rc=$?; tail -3 $O/pytest_sched.log; exit $rc
