# round 5 GPU pass g: the f1 forward epilogue on the running base (no per-tile max pass unless a logit
# passes the running max by 2^20): parity tests, f1_ab standalone (plain and right after GEMM load)
# against the previous library (verl_amd/lib/ab/lib_head.so), interleaved; then the bench default
set -o pipefail
O=gpurun_out/r05/g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_linear_logprob_gpu.py tests/test_reference_protocol_gpu.py tests/test_golden_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest FAILED"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for pre in 0 400; do
    VERL_AMD_LIB=verl_amd/lib/ab/lib_head.so timeout -k 10 200 python tools/f1_ab.py --tag head --iters 4 --pre-gemm-ms $pre >> $O/f1_ab.jsonl 2>> $O/f1_ab.err || { echo "f1 head FAILED"; tail $O/f1_ab.err; exit 1; }
    timeout -k 10 200 python tools/f1_ab.py --tag runbase --iters 4 --pre-gemm-ms $pre >> $O/f1_ab.jsonl 2>> $O/f1_ab.err || { echo "f1 new FAILED"; tail $O/f1_ab.err; exit 1; }
  done
done
python3 -c "
import json
for l in open('$O/f1_ab.jsonl'):
    d=json.loads(l); print(d['tag'], d['pre_gemm_ms'], d['ms_median'], d['tflops'], d['max_dlp_vs_unfused'], d['max_dent_vs_unfused'])"
bash tools/gpu_ab.sh f1_runbase 2 "VERL_AMD_LIB=verl_amd/lib/ab/lib_head.so" "" > $O/bench_ab.txt 2>&1 || { echo "AB FAILED"; cat $O/bench_ab.txt; exit 1; }
cat $O/bench_ab.txt
for i in 1 2 3 4; do python -c "
import json;d=json.loads([l for l in open('gpurun_out/ab_f1_runbase/run_$i.json') if l.startswith('{')][-1]);f=d.get('roofline_f1') or {}
print($i, d['value'], f.get('avg_launch_us'), f.get('frac'))"; done
