# round 5 GPU pass e: (1) flash forward without the per-block row max / cross-lane exchanges in the
# steady state (pass-0 fast path): attention parity tests, then attn_ab against the previous library
# (verl_amd/lib/ab/lib_base.so), interleaved; (2) the no-grad f1 as ONE launch over all micro-batches
# (--f1-concat 1) vs 4 launches after the backbones, interleaved bench A/B
set -o pipefail
O=gpurun_out/r05/e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_attention_gpu.py tests/test_linear_logprob_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest FAILED"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  VERL_AMD_LIB=verl_amd/lib/ab/lib_base.so timeout -k 10 200 python tools/attn_ab.py --tag base >> $O/attn_ab.jsonl 2>> $O/attn_ab.err || { echo "attn base FAILED"; tail $O/attn_ab.err; exit 1; }
  timeout -k 10 200 python tools/attn_ab.py --tag fastpath >> $O/attn_ab.jsonl 2>> $O/attn_ab.err || { echo "attn new FAILED"; tail $O/attn_ab.err; exit 1; }
done
cut -c1-220 $O/attn_ab.jsonl
bash tools/gpu_ab.sh f1_concat 2 "" "--f1-concat 1" > $O/f1_concat_ab.txt 2>&1 || { echo "AB FAILED"; cat $O/f1_concat_ab.txt; exit 1; }
cat $O/f1_concat_ab.txt
for i in 1 2 3 4; do python -c "
import json;d=json.loads([l for l in open('gpurun_out/ab_f1_concat/run_$i.json') if l.startswith('{')][-1]);f=d.get('roofline_f1') or {}
print($i, d['value'], f.get('avg_launch_us'), f.get('launches'), f.get('frac'))"; done
