# round 5 GPU pass ad: f1 sweep variants, interleaved at the bench shape — at1 (the committed
# product: LDS-DMA by global_load_lds between the K-halves), bufload (the same, through buffer
# resources: 32-bit offsets, bounds by record count), defer (bufload + the tile epilogue deferred
# into the next tile's first K-step, column by column with the MFMAs); then the sweep users' parity
# tests on each new variant
set -o pipefail
O=gpurun_out/r05/ad
mkdir -p $O
for i in 1 2 3; do
  for v in at1 bufload defer; do
    VERL_AMD_LIB=verl_amd/lib/ab/libverl_amd_$v.so timeout -k 10 120 python tools/f1_ab.py --tag $v >> $O/f1_variants_ab.jsonl 2>> $O/f1_ab.err || { echo "$v FAILED"; tail -20 $O/f1_ab.err; exit 1; }
  done
done
python -c "
import json
for l in open('$O/f1_variants_ab.jsonl'): d=json.loads(l); print(d['tag'], d['ms_median'], d['max_dlp_vs_unfused'], d['max_dent_vs_unfused'])"
for v in bufload defer; do
  VERL_AMD_LIB=verl_amd/lib/ab/libverl_amd_$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_linear_logprob_gpu.py tests/test_model_ops_gpu.py tests/test_reference_protocol_gpu.py tests/test_fused_backends_gpu.py > $O/pytest_$v.log 2>&1 || { echo "TESTS $v FAILED"; tail -30 $O/pytest_$v.log; exit 1; }
  echo $v; tail -1 $O/pytest_$v.log
done
