# round 4 GPU pass o (flash LDS-DMA staging default): the -m gpu suite (incl. the W = 8 gloo rehearsal, JSON + logs kept under
# gpurun_out/r04/rehearsal), smoke(), one default bench line
set -o pipefail
O=gpurun_out/r04
mkdir -p $O
export VA_REHEARSAL_OUT=$O/rehearsal
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 700 --timeout-method thread > $O/pytest_gpu_o.log 2>&1 || { echo "pytest FAILED"; tail -60 $O/pytest_gpu_o.log; exit 1; }
tail -3 $O/pytest_gpu_o.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_o.log 2>&1 || { echo "smoke FAILED"; tail -30 $O/smoke_o.log; exit 1; }
tail -2 $O/smoke_o.log
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --out $O/bench_o_default.json > $O/bench_o_default.log 2>&1 || { echo "bench default FAILED"; tail -30 $O/bench_o_default.log; exit 1; }
head -c 1500 $O/bench_o_default.json; echo
