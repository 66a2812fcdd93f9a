# round 5 GPU pass r: torch_functional log-prob family drop-ins
set -o pipefail
O=gpurun_out/r05/r
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_torch_functional_gpu.py -v --timeout 120 --timeout-method thread > $O/pytest_tf.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|Error|assert" $O/pytest_tf.log | tail -30
exit $rc
