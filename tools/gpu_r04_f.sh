# round 4 GPU pass f: the actor / critic / Qwen2-VL / bench-config / linear-logprob tests after the
# reference labels at masked positions
set -o pipefail
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_actor_gpu.py tests/test_critic_gpu.py tests/test_qwen2_vl_gpu.py tests/test_bench_config_parity_gpu.py tests/test_linear_logprob_gpu.py tests/test_loss_segments_gpu.py -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu_f.log 2>&1 || { echo "pytest FAILED"; grep -E "Error|assert|FAILED" $O/pytest_gpu_f.log | head -30; tail -40 $O/pytest_gpu_f.log; exit 1; }
tail -3 $O/pytest_gpu_f.log
