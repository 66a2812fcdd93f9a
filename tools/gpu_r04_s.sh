# round 4 GPU pass s: the no-grad old-logp pass's micro-batch (log_prob_micro_batch_size_per_gpu;
# per-row results are independent of it) at 128 (bench default) / 256 / 512 responses, interleaved;
# plus the realistic-length variant at the defaults
set -o pipefail
O=gpurun_out/r04/lpmicro
mkdir -p $O
for r in 1 2; do
  for m in 128 256 512; do
    timeout -k 10 400 python bench.py --steps 3 --warmup 1 --logprob-micro $m --no-cpu-baseline --no-kernel-timing --out $O/m${m}_r$r.json > $O/m${m}_r$r.log 2>&1 || { echo "bench m=$m FAILED"; tail -20 $O/m${m}_r$r.log; exit 1; }
    python -c "import json;d=json.load(open('$O/m${m}_r$r.json'));print($m, d['value'], d['ms_per_step'], d.get('peak_hbm_gb'))"
  done
done
timeout -k 10 600 python bench.py --responses realistic --no-cpu-baseline --out $O/realistic.json > $O/realistic.log 2>&1 || { echo "realistic FAILED"; tail -20 $O/realistic.log; exit 1; }
python -c "import json;d=json.load(open('$O/realistic.json'));print('realistic', d['value'], d['ms_per_step'], d.get('peak_hbm_gb'))"
