#!/bin/bash
# same-box A/B of the attention kernels: the library at $1 (old) vs the in-tree one (new), interleaved twice
set -u
O=gpurun_out/attnab
mkdir -p $O
for r in 1 2; do
  VERL_AMD_LIB=$1 timeout -k 10 300 python tools/attn_bwd_ab.py > $O/old$r.log 2>&1 || exit $?
  timeout -k 10 300 python tools/attn_bwd_ab.py > $O/new$r.log 2>&1 || exit $?
done
grep -h '"case"' $O/old1.log $O/old2.log | sed 's/^/old /'
grep -h '"case"' $O/new1.log $O/new2.log | sed 's/^/new /'
