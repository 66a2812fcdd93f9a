#!/bin/bash
# Headline-bench A/B of the backbone input-gradient GEMM layout (kernels.input_grad):
# plain "NN" product vs the transposed-weight "TN" product, interleaved on one box
set -u
O=gpurun_out/dgrad_ab
mkdir -p $O
i=0
for L in nn tn nn tn; do
  i=$((i + 1))
  VERL_AMD_DGRAD_LAYOUT=$L timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline \
    --out $O/$L$i.json > $O/$L$i.log 2>&1 || exit $?
  python3 -c "import json;d=json.load(open('$O/$L$i.json'));print('$L', d['value'], d['ms_per_step'])"
done
