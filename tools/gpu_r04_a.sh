# round 4, first GPU pass: f1 forward old/new library A/B (sweep refactor), the fused backward vs
# its composition, then the whole -m gpu suite (incl. the W = 8 gloo rehearsal, whose JSON lines are
# kept under gpurun_out/r04/rehearsal) and smoke()
set -o pipefail
O=gpurun_out/r04
mkdir -p $O
for i in 1 2; do
  VERL_AMD_LIB_AB=1 VERL_AMD_LIB=scratch/ab/libverl_amd_r03.so timeout -k 10 120 python tools/f1_ab.py --tag r03 >> $O/f1_fwd_refactor_ab.jsonl 2>>$O/f1_ab.err || { echo "f1_ab r03 FAILED"; tail $O/f1_ab.err; exit 1; }
  timeout -k 10 120 python tools/f1_ab.py --tag r04 >> $O/f1_fwd_refactor_ab.jsonl 2>>$O/f1_ab.err || { echo "f1_ab r04 FAILED"; tail $O/f1_ab.err; exit 1; }
done
cat $O/f1_fwd_refactor_ab.jsonl
timeout -k 10 300 python tools/f1_bwd_ab.py > $O/f1_bwd_ab.json 2>$O/f1_bwd_ab.err || { echo "f1_bwd_ab FAILED"; tail -30 $O/f1_bwd_ab.err; exit 1; }
cat $O/f1_bwd_ab.json
export VA_REHEARSAL_OUT=$O/rehearsal
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 700 --timeout-method thread > $O/pytest_gpu_a.log 2>&1 || { echo "pytest FAILED"; tail -60 $O/pytest_gpu_a.log; exit 1; }
tail -3 $O/pytest_gpu_a.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_a.log 2>&1 || { echo "smoke FAILED"; tail -30 $O/smoke_a.log; exit 1; }
tail -2 $O/smoke_a.log
