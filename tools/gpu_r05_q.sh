# round 5 GPU pass q: drop-ins for the reference's fused lm_head backends (linear_cross_entropy with
# reduction / vocab tensor parallelism, FusedLinearForPPO) + the f1 tests the shard offset touches
set -o pipefail
O=gpurun_out/r05/q
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_fused_backends_gpu.py tests/test_linear_logprob_gpu.py tests/test_kats_gpu.py -v --timeout 300 --timeout-method thread > $O/pytest_fused_backends.log 2>&1; rc=$?
grep -E "PASSED|FAILED|SKIPPED|ERROR|passed|failed" $O/pytest_fused_backends.log | tail -60
exit $rc
