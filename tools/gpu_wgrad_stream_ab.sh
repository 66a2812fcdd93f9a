#!/bin/bash
# side-stream weight gradients: parity tests, then an interleaved same-box bench A/B (0 = one stream)
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/wgs
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_wgrad_stream_gpu.py tests/test_bench_config_parity_gpu.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for ws in ${ORDER:-1 0 1 0}; do
  i=$((${i:-0}+1))
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --wgrad-stream $ws \
    --out $O/bench_ws${ws}_$i.json > $O/bench_ws${ws}_$i.log 2>&1 || exit $?
  python -c "import json;d=json.load(open('$O/bench_ws${ws}_$i.json'));print('ws=$ws', d['value'], d['ms_per_step'], d['config']['peak_hbm_gb'])"
done
