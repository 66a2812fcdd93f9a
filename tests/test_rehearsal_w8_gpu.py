"""bench.py at world size 8 on one GPU (missing #3).

The driver's 8-GPU scaling run is the bench's first contact with W = 8. This test runs the same
command first, with the 8 ranks sharing one MI355X over gloo (RCCL refuses two ranks on one
device): 8 prompts x n = 8 responses x 256 tokens split into 1 prompt (8 responses) per rank,
compute micro-batch capped at the rank's shard, ZeRO shards padded to 64 W elements. Three modes:
strong scaling (groups intact), ``--balance`` (Karmarkar-Karp, groups split: the cross-rank GRPO
exchange runs) and ``--zero 1`` (reduce-scatter + all-gather of the sharded masters). Each must
  * see world size 8 and finish with every rank's weights, masters and global metrics identical
    (bench's replica check);
  * equal the same global batch at W = 1 up to the rounding of per-rank bf16 gradients: the grad
    norm within 0.5 % (this catches a missing or doubled 1/W), and the fp32 master update (after -
    before, a strided sample over all parameters) with cosine >= 0.99 and relative L2 error <= 10 %
    of the W = 1 update (AdamW's first steps move each weight by ~lr sign(g): the error is the
    ~0.1 % of weights whose tiny gradients flip sign under the bf16 rounding).
The reference gets this W-independence from FSDP's mean reduction over one sharded parameter set
(fsdp_workers.py:340-347, 370-405) and the DP_COMPUTE_PROTO chunking (decorator.py:375-385)."""

import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--prompts", "8", "--response-len", "256", "--prompt-len", "128", "--steps", "1", "--warmup", "1",
         "--no-cpu-baseline", "--no-kernel-timing"]


def _bench(tmp, name, gpus, extra=(), scratch=None):
    out, dump = os.path.join(tmp, f"bench_rehearsal_{name}_gloo.json"), os.path.join(scratch or tmp, f"{name}.npz")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["VA_DIST_BACKEND"] = "gloo"
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), *SMALL, *extra,
           "--out", out, "--dump-state", dump]
    print("running:", " ".join(cmd[2:]), flush=True)
    res = subprocess.run(cmd, env=env, cwd=ROOT, timeout=600, capture_output=True, text=True)
    with open(os.path.join(tmp, f"{name}.log"), "w") as f:
        f.write(res.stderr)
    tb = res.stderr.find("Traceback")
    assert res.returncode == 0, res.stderr[tb : tb + 3000] if tb >= 0 else res.stderr[-4000:]
    rec = json.loads(open(out).read())
    print(name, {k: rec[k] for k in ("value", "ms_per_step", "world_seen", "replicas_identical")}, flush=True)
    return rec, np.load(dump)


@pytest.mark.gpu
def test_bench_world8_gloo_rehearsal_matches_world1(tmp_path):
    import gc

    import torch

    # the 8 ranks share this GPU with the test process: hand back what earlier tests left cached
    gc.collect()
    torch.cuda.empty_cache()
    tmp = os.environ.get("VA_REHEARSAL_OUT") or str(tmp_path)  # keep the JSON lines and logs when asked
    os.makedirs(tmp, exist_ok=True)
    r1, d1 = _bench(tmp, "w1", 1, scratch=str(tmp_path))
    u1 = d1["masters"].astype(np.float64) - d1["masters_init"]
    g1 = float(d1["actor__grad_norm"].reshape(-1)[-1])
    assert np.linalg.norm(u1) > 0
    for name, extra in (("w8_strong", ()), ("w8_balance", ("--balance",)), ("w8_zero", ("--zero", "1"))):
        rec, d8 = _bench(tmp, name, 8, extra, scratch=str(tmp_path))
        assert rec["world_seen"] == 8 and rec["n_gpus"] == 8
        assert rec["replicas_identical"] is True, rec["replica_check"]
        assert rec["config"]["responses_per_gpu"] == 8
        assert rec["config"]["groups_split_over_ranks"] == (name == "w8_balance")
        assert np.array_equal(d8["masters_init"], d1["masters_init"])  # rank 0's init broadcast
        g8 = float(d8["actor__grad_norm"].reshape(-1)[-1])
        assert abs(g8 - g1) <= 5e-3 * g1, (name, g8, g1)
        u8 = d8["masters"].astype(np.float64) - d8["masters_init"]
        cos = float(u1 @ u8 / (np.linalg.norm(u1) * np.linalg.norm(u8)))
        rel = float(np.linalg.norm(u8 - u1) / np.linalg.norm(u1))
        print(name, "grad_norm", g8, "vs", g1, "update cos", cos, "rel", rel, flush=True)
        assert cos >= 0.99 and rel <= 0.1, (name, cos, rel)
