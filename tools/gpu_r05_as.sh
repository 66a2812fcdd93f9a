# round 5 GPU pass as: full GPU suite + smoke() + the driver bench command at the ABI-9 head
set -o pipefail
O=gpurun_out/r05/as
mkdir -p $O
export VA_REHEARSAL_OUT=$O/rehearsal
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest FAILED"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke FAILED"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --out $O/bench.json > $O/bench.log 2>&1 || { echo "bench FAILED"; tail -30 $O/bench.log; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['frac'], r.get('launch_us_min_median_max'), d['roofline_hbm']['frac'], d['cpu_baseline']['value'])"
