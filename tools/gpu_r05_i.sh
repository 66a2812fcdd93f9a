# round 5 GPU pass i: the q|k|v bias gradient by va_column_sum — its tests, then an interleaved bench
# A/B against torch's dy.sum(0) (VERL_AMD_BIAS_SUM=torch)
set -o pipefail
O=gpurun_out/r05/i
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_model_ops_gpu.py tests/test_abi.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest FAILED"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_ab.sh bias_sum 2 "VERL_AMD_BIAS_SUM=torch" "" > $O/bias_sum_ab.txt 2>&1 || { echo "AB FAILED"; cat $O/bias_sum_ab.txt; exit 1; }
cat $O/bias_sum_ab.txt
