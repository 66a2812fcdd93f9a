# round 5 GPU pass am: the fused gate|up + SwiGLU's LDS-staged stores as committed (16-B alignment
# checks): the model-ops and linear_logprob parity tests and the default bench
set -o pipefail
O=gpurun_out/r05/am
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_model_ops_gpu.py tests/test_linear_logprob_gpu.py tests/test_abi.py > $O/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --out $O/bench.json > $O/bench.log 2>&1 || { echo "bench FAILED"; tail -20 $O/bench.log; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
