# round 5 GPU pass j: the full GPU suite and smoke() at HEAD (column-sum second stage widened)
set -o pipefail
O=gpurun_out/r05/j
mkdir -p $O
export VA_REHEARSAL_OUT=$O/rehearsal
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest FAILED"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke FAILED"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
