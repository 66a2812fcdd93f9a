# round 5 GPU pass d: the no-grad pass's fused lm_head launched after all backbones (f1 clock
# recovery) — its parity test, then an interleaved bench A/B: after-backbone (default) vs per
# micro-batch vs the unfused no-grad pass (hipBLASLt lm_head GEMM + logprob_entropy_fwd)
set -o pipefail
O=gpurun_out/r05/d
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_linear_logprob_gpu.py -x -q -k "no_grad" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest FAILED"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_ab.sh f1_order 2 "" "--f1-after-backbone 0" "--fused-no-grad 0" > $O/f1_order_ab.txt 2>&1 || { echo "AB FAILED"; cat $O/f1_order_ab.txt; exit 1; }
cat $O/f1_order_ab.txt
for i in 1 2 3 4 5 6; do python -c "
import json;d=json.loads([l for l in open('gpurun_out/ab_f1_order/run_$i.json') if l.startswith('{')][-1]);r=d['roofline'];f=d.get('roofline_f1') or {}
print($i, d['value'], r['kernel'], r['frac'], f.get('avg_launch_us'), f.get('frac'))"; done
