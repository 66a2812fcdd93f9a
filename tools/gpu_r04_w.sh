# round 4 GPU pass w: the -m gpu suite + smoke() at HEAD (after the dK/dV row-constant fix)

set -o pipefail
O=gpurun_out/r04
mkdir -p $O
export VA_REHEARSAL_OUT=$O/rehearsal_w
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 700 --timeout-method thread > $O/pytest_gpu_w.log 2>&1 || { echo "pytest FAILED"; tail -40 $O/pytest_gpu_w.log; exit 1; }
tail -2 $O/pytest_gpu_w.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_w.log 2>&1 || { echo "smoke FAILED"; tail -20 $O/smoke_w.log; exit 1; }
tail -1 $O/smoke_w.log

