# round 5 GPU pass p: hand-derived / closed-form KATs on the HIP kernels (policy loss, agg, KL,
# whitening, GRPO, log-prob + entropy fwd/bwd, fused lm_head fwd/bwd)
set -o pipefail
O=gpurun_out/r05/p
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kats_gpu.py -v --timeout 120 --timeout-method thread > $O/pytest_kats.log 2>&1; rc=$?
tail -40 $O/pytest_kats.log
exit $rc
