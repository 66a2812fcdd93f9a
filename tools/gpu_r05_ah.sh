# round 5 GPU pass ah: f1 vocab splits after the staging rework (VERL_AMD_LINEAR_LOGPROB_SPLITS),
# interleaved at the bench shape
set -o pipefail
O=gpurun_out/r05/ah
mkdir -p $O
for i in 1 2; do
  for sp in 4 6 8 12 16; do
    VERL_AMD_LINEAR_LOGPROB_SPLITS=$sp timeout -k 10 120 python tools/f1_ab.py --tag splits$sp >> $O/f1_splits_ab.jsonl 2>> $O/f1_ab.err || { echo "$sp FAILED"; tail -20 $O/f1_ab.err; exit 1; }
  done
done
python -c "
import json
for l in open('$O/f1_splits_ab.jsonl'): d=json.loads(l); print(d['tag'], d['ms_median'])"
