#!/bin/bash
# GPU box: the whole -m gpu suite in one process, then smoke().
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/t_full.log 2>&1
rc=$?; echo "[pytest -m gpu] rc=$rc"; tail -3 gpurun_out/t_full.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "[smoke] rc=$rc"; tail -2 gpurun_out/smoke.log
exit $rc
