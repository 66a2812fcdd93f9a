"""bench.py's multi-rank launcher, on CPU (gloo): ``--gpus N`` without a launcher starts
torch.distributed.run as a child with N ranks, every rank sees world size N, and a failing rank
makes the whole command exit non-zero."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n, extra_env=None, extra_args=()):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update({"VA_DIST_BACKEND": "gloo", "OMP_NUM_THREADS": "1"})
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--launcher-check",
                           *extra_args], capture_output=True, text=True, env=env, timeout=300, cwd=ROOT)


@pytest.mark.parametrize("n", [2, 3])
def test_launcher_spawns_n_ranks(n):
    res = _run(n)
    assert res.returncode == 0, res.stderr[-2000:]
    lines = [json.loads(x) for x in res.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, res.stdout  # rank 0 only
    rec = lines[0]
    assert rec["n_gpus"] == n and rec["world_seen"] == n
    assert rec["rank_sum"] == n * (n + 1) / 2  # every rank joined the all-reduce


def test_launcher_propagates_rank_failure():
    res = _run(2, {"VA_BENCH_FAIL_RANK": "1"})
    assert res.returncode != 0


def test_world_size_mismatch_is_an_error():
    # under an explicit single-process "launcher" env, --gpus 2 must not silently run one rank
    res = _run(2, {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert res.returncode != 0


def test_replica_check_passes_when_ranks_agree_and_fails_when_one_rank_differs():
    """the end-of-run replica check (utils/replica_check.py) runs through the
    same launcher; equal replicas report replicas_identical, one rank's weight changed after the
    update makes the command exit non-zero."""
    res = _run(2)
    assert res.returncode == 0, res.stderr[-2000:]
    rec = [json.loads(x) for x in res.stdout.splitlines() if x.startswith("{")][0]
    assert rec["replicas_identical"] is True and rec["weights_equal"] and rec["metrics_equal"]
    bad = _run(2, {"VA_BENCH_PERTURB_RANK": "1"})
    assert bad.returncode != 0
    rec = [json.loads(x) for x in bad.stdout.splitlines() if x.startswith("{")][0]
    assert rec["replicas_identical"] is False and not rec["weights_equal"] and rec["metrics_equal"]


def test_bits_checksum_is_order_independent_and_position_sensitive():
    import torch

    from verl_amd.utils.replica_check import bits_checksum

    g = torch.Generator().manual_seed(0)
    a = torch.randn(1000, generator=g)
    b = a.clone()
    b[[3, 7]] = b[[7, 3]]  # swapped pair
    c = a.clone()
    c[5] = torch.nextafter(c[5], torch.tensor(10.0))  # one ulp
    x = bits_checksum([a, a.to(torch.bfloat16)])
    assert int(x) == int(bits_checksum([a, a.to(torch.bfloat16)]))
    assert int(x) != int(bits_checksum([b, a.to(torch.bfloat16)]))
    assert int(x) != int(bits_checksum([c, a.to(torch.bfloat16)]))
