# bench.py at W = 8 on one GPU (gloo), three modes, plus the same global batch at W = 1
# (VERDICT r3 next #1); outputs under gpurun_out/r04/, copied to profiles/r04/ afterwards.
set -o pipefail
export VA_DIST_BACKEND=gloo
O=gpurun_out/r04
mkdir -p $O
SMALL="--prompts 8 --response-len 256 --prompt-len 128 --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 python -u bench.py --gpus 1 $SMALL --out $O/bench_rehearsal_w1_gloo.json --dump-state $O/rehearsal_w1.npz > $O/rehearsal_w1.log 2>&1 || { echo "FAIL w1"; tail -30 $O/rehearsal_w1.log; exit 1; }
echo "OK w1"
for mode in strong balance zero; do
  extra=""
  [ $mode = balance ] && extra="--balance"
  [ $mode = zero ] && extra="--zero 1"
  timeout -k 10 420 python -u bench.py --gpus 8 $SMALL $extra --out $O/bench_rehearsal_w8_gloo_$mode.json --dump-state $O/rehearsal_w8_$mode.npz > $O/rehearsal_w8_$mode.log 2>&1 || { echo "FAIL $mode"; tail -40 $O/rehearsal_w8_$mode.log; exit 1; }
  echo "OK $mode"; head -c 400 $O/bench_rehearsal_w8_gloo_$mode.json; echo
done
