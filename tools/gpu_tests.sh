#!/bin/bash
# GPU parity tests only (one process), optional pytest -k filter as $1
set -u
mkdir -p gpurun_out
K=${1:-}
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider -k "$K" > gpurun_out/tests.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests.log 2>&1
fi
rc=$?; echo "rc=$rc" >> gpurun_out/tests.log; tail -30 gpurun_out/tests.log; exit $rc
