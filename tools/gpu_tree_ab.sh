#!/bin/bash
# Same-box headline-bench A/B of two trees: $1 = an older checkout (with its built library),
# against this tree; interleaved A B A B
set -u
OLD=$1
O=$PWD/gpurun_out/tree_ab
mkdir -p $O
i=0
for T in old new old new; do
  i=$((i + 1))
  D=$PWD; [ $T = old ] && D=$OLD
  (cd $D && timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --out $O/$T$i.json > $O/$T$i.log 2>&1) || exit $?
  python3 -c "import json;d=json.load(open('$O/$T$i.json'));print('$T', d['value'], d['ms_per_step'])"
done
