# round 5 GPU pass an: the fused backward's dlogits stores through a wave-private LDS scratch (whole
# 16-B pieces of token rows) vs direct 8-byte stores (HEAD build): linear_logprob / fused-backend
# parity tests, then the pass-level A/B (tools/f1_bwd_ab.py) and the fused-kernel bench, interleaved
set -o pipefail
O=gpurun_out/r05/an
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_linear_logprob_gpu.py tests/test_fused_backends_gpu.py tests/test_reference_protocol_gpu.py > $O/pytest.log 2>&1 || { echo "TESTS FAILED"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  VERL_AMD_LIB=verl_amd/lib/ab/libverl_amd_base.so VERL_AMD_LIB_AB=1 timeout -k 10 400 python tools/f1_bwd_ab.py >> $O/f1_bwd_base.jsonl 2>> $O/bwd.err || { echo "base FAILED"; tail -20 $O/bwd.err; exit 1; }
  timeout -k 10 400 python tools/f1_bwd_ab.py >> $O/f1_bwd_new.jsonl 2>> $O/bwd.err || { echo "new FAILED"; tail -20 $O/bwd.err; exit 1; }
done
python -c "
import json
for v in ('base','new'):
    for l in open('$O/f1_bwd_'+v+'.jsonl'):
        d=json.loads(l); print(v, d.get('fused_dlogits_ms'), d.get('fused_pass_split9504_ms'), d.get('unfused_pass_ms'))"
run() { local tag=$1; shift; timeout -k 10 400 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --fused-kernels 1 --out $O/bench_$tag.json "$@" > $O/bench_$tag.log 2>&1 || { echo "$tag FAILED"; tail -20 $O/bench_$tag.log; exit 1; }; python -c "import json;d=json.load(open('$O/bench_$tag.json'));print('$tag', d['value'], d['ms_per_step'], d['config']['peak_hbm_gb'])"; }
VERL_AMD_LIB=verl_amd/lib/ab/libverl_amd_base.so VERL_AMD_LIB_AB=1 run base_fused
run new_fused
