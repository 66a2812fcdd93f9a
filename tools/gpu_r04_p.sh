# NOTE: the VA_F1_PRIO variants were measured from a working-tree patch and not kept.
# round 4 GPU pass p: f1 forward with s_setprio (VA_F1_PRIO builds: 1 = priority 1 around each
# step's MFMA cluster, 2 = waves 4-7 at priority 1 for the whole sweep) vs the product build, interleaved
set -o pipefail
O=gpurun_out/r04/f1_prio
mkdir -p $O
for r in 1 2; do
  timeout -k 10 120 python tools/f1_ab.py --tag base >> $O/time.jsonl || exit 1
  for v in 1 2; do
    VERL_AMD_LIB=verl_amd/lib/ab/libverl_amd_prio$v.so timeout -k 10 120 python tools/f1_ab.py --tag prio$v >> $O/time.jsonl || exit 1
  done
done
python -c "
import json
for l in open('$O/time.jsonl'):
    d=json.loads(l); print(d['tag'], d['ms_median'], d['max_dlp_vs_unfused'])"
