# round 5 GPU pass ab: f1 staging position — branch-free LDS-DMA staging issued before the step's
# MFMAs (at0) or between its two K-halves (at1) vs the current sweep (base), interleaved
set -o pipefail
O=gpurun_out/r05/ab
mkdir -p $O
for i in 1 2 3; do
  for v in base at0 at1; do
    VERL_AMD_LIB=verl_amd/lib/ab/libverl_amd_$v.so timeout -k 10 120 python tools/f1_ab.py --tag $v >> $O/f1_stage_at_ab.jsonl 2>> $O/f1_ab.err || { echo "$v FAILED"; tail -20 $O/f1_ab.err; exit 1; }
  done
done
python -c "
import json
for l in open('$O/f1_stage_at_ab.jsonl'): d=json.loads(l); print(d['tag'], d['ms_median'], d['max_dlp_vs_unfused'])"
