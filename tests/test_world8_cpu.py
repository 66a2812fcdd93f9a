"""World size 8 on CPU with the RCCL branches forced.

The driver's 8-GPU scaling run is the first time the data-parallel path meets 8 ranks on RCCL.
Here 8 gloo ranks run the same code with ``tests/_nccl_emulation.py`` active, so every branch
that only RCCL reaches executes at W = 8 first: the AVG bucket all-reduces of the gradient
managers, the ZeRO reduce-scatter (AVG) of buckets padded to 64 W elements and the all-gather of
the bf16 shards into the flat weight buffers, the comm-device staging of the advantage exchange,
the metric reduction and the replica check. Each is checked against a single-process computation
of the same mini-batch (the reference's FSDP mean semantics, fsdp_workers.py:340-347, 370-405;
DP_COMPUTE_PROTO chunk order, decorator.py:375-408), and the emulated calls are counted so the test
fails if a branch silently fell back to the gloo path."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

WORLD = 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(seed=0, width=40):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(6, width), torch.nn.Tanh(), torch.nn.Linear(width, 3))


def _data(world):
    g = torch.Generator().manual_seed(5)
    return [torch.randn(4, 6, generator=g) for _ in range(world * 2)]


def _train(mgr, mod, opt, xs, rank, step, max_norm):
    """One mini-batch: 2 micro-batches per rank (loss / grad-accum), sync on the last, clip, AdamW."""
    mgr.zero_grad()
    mine = xs[rank * 2 : rank * 2 + 2]
    for i, x in enumerate(mine):
        if i == len(mine) - 1:
            mgr.begin_sync()
        (mod(x.bfloat16() + step).float().square().mean() / len(mine)).backward()
    mgr.finish_sync()
    norm = mgr.clip_grad_norm_(max_norm)
    opt.step()
    mgr.after_step()
    return norm


def _worker(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    from tests import _nccl_emulation as emu

    emu.enable()
    from verl_amd.utils import comm
    from verl_amd.utils.replica_check import replica_check
    from verl_amd.workers.grad_sync import GradBucketReducer, MixedPrecisionParams, ShardedMixedPrecisionParams

    assert comm.device_backend() and comm.world() == world

    # ---------------------------------------------------------------- replicated bf16 + fp32 masters
    xs = _data(world)
    a = _model()
    rep = MixedPrecisionParams(a, bucket_bytes=512)
    assert len(rep.buckets) > 1 and rep._use_avg
    opt_a = torch.optim.AdamW(rep.optimizer_params(), lr=1e-2, weight_decay=0.01, foreach=False)
    # single-process reference of the same mini-batch: all 2W micro-batches, loss / 2W each
    # (grad-accum 2 per rank, then the mean over W ranks), same bf16 forward / backward
    one = _model()
    one_mgr = MixedPrecisionParams(one, bucket_bytes=512, process_group=None)
    one_mgr.world = 1  # accumulate locally only (this process is one of 8; the reference is W = 1)
    one_mgr._use_avg = False
    one_opt = torch.optim.AdamW(one_mgr.optimizer_params(), lr=1e-2, weight_decay=0.01, foreach=False)
    before = dict(emu.CALLS)
    for step in range(2):
        n8 = _train(rep, a, opt_a, xs, rank, step, 0.5)
        one_mgr.zero_grad()
        for x in xs:
            (one(x.bfloat16() + step).float().square().mean() / 2 / world).backward()
        one_mgr.after_backward()
        n1 = one_mgr.clip_grad_norm_(0.5)
        one_opt.step()
        one_mgr.after_step()
        # fp32 mean of per-rank bf16 gradient sums vs one fp32 sum: reduction-order rounding only
        assert torch.allclose(n8, n1, rtol=1e-3), (step, float(n8), float(n1))
        for m8, m1 in zip(rep.optimizer_params(), one_mgr.optimizer_params(), strict=True):
            assert torch.allclose(m8, m1, atol=2e-4, rtol=0), step
    assert emu.CALLS["all_reduce_avg"] - before.get("all_reduce_avg", 0) >= 2 * len(rep.buckets)
    rc = replica_check(a, rep, {"actor/grad_norm": [float(n8)]}, ["actor/grad_norm"], 0.0)
    assert rc["replicas_identical"] and rc["masters_checked"] and rc["world"] == world, rc

    # ---------------------------------------------------------------- ZeRO shards == replicated
    b = _model()
    shd = ShardedMixedPrecisionParams(b, bucket_bytes=512)
    c = _model()
    rep2 = MixedPrecisionParams(c, bucket_bytes=512)
    assert shd._use_avg and len(shd.buckets) > 1
    for bk, s in zip(shd.buckets, shd.shards, strict=True):
        assert bk.buf.numel() % (64 * world) == 0 and s.numel() * world == bk.buf.numel()
    opt_b = torch.optim.AdamW(shd.optimizer_params(), lr=1e-2, weight_decay=0.01, foreach=False)
    opt_c = torch.optim.AdamW(rep2.optimizer_params(), lr=1e-2, weight_decay=0.01, foreach=False)
    before = dict(emu.CALLS)
    for step in range(3):
        nb = _train(shd, b, opt_b, xs, rank, step, 0.5)
        nc = _train(rep2, c, opt_c, xs, rank, step, 0.5)
        assert torch.allclose(nb, nc, rtol=1e-5), (step, float(nb), float(nc))
        for p, q in zip(b.parameters(), c.parameters(), strict=True):
            assert p.dtype == q.dtype == torch.bfloat16
            assert torch.allclose(p.float(), q.float(), atol=1e-2, rtol=0), step
    got = emu.CALLS
    assert got["reduce_scatter_tensor_avg"] - before.get("reduce_scatter_tensor_avg", 0) == 3 * len(shd.buckets)
    assert got["all_gather_into_tensor"] - before.get("all_gather_into_tensor", 0) == 3 * len(shd.buckets)
    rc = replica_check(b, shd, {"actor/grad_norm": [float(nb)]}, ["actor/grad_norm"], 0.0)
    assert rc["replicas_identical"] and rc["masters_sharded"], rc

    # ---------------------------------------------------------------- fp32 reducer (no mixed precision)
    d = _model()
    red = GradBucketReducer(d.parameters(), bucket_bytes=256)
    assert red._use_avg
    red.zero_grad()
    for i, x in enumerate(xs[rank * 2 : rank * 2 + 2]):
        if i == 1:
            red.begin_sync()
        (d(x).square().mean() / 2).backward()
    red.finish_sync()
    ref = _model()
    for x in xs:
        (ref(x).square().mean() / (2 * world)).backward()
    for p, q in zip(d.parameters(), ref.parameters(), strict=True):
        assert torch.allclose(p.grad, q.grad, atol=1e-6)

    # ---------------------------------------------------------------- exchanges of the step
    from verl_amd.trainer.ppo.dp_algos import agg_loss_dp, check_groups_intact, gather_row_scores
    from verl_amd.trainer.ppo.trainer_step import reduce_metrics_dp

    rows = list(range(3 * rank, 3 * rank + 3))
    uids = np.array([f"g{i // 2}" for i in rows], dtype=object)
    s_all, _, _, off = gather_row_scores(torch.tensor([float(i) for i in rows]), None, uids, None)
    assert off == 3 * rank and s_all.tolist() == [float(i) for i in range(3 * world)]
    assert not check_groups_intact(uids)
    assert check_groups_intact(np.array([f"r{rank}-{i}" for i in range(4)], dtype=object))
    g = torch.Generator().manual_seed(7)
    x = torch.randn(world * 5, 9, generator=g)
    mask = (torch.rand(world * 5, 9, generator=g) > 0.3).long()
    mask[:, 0] = 1
    mine = slice(rank * 5, (rank + 1) * 5)
    from oracle import reference_ops as oref

    for mode in ("token-mean", "seq-mean-token-sum", "seq-mean-token-mean", "seq-mean-token-sum-norm"):
        got_l = agg_loss_dp(x[mine], mask[mine], mode)
        assert torch.allclose(got_l, oref.agg_loss(x, mask, mode).float(), rtol=1e-6, atol=1e-6), mode
    red_m = reduce_metrics_dp({"actor/pg_loss": [float(rank), float(rank) + 1], "actor/x_max": [float(rank)],
                               "actor/y_min": [float(rank)]})
    assert red_m["actor/pg_loss"] == pytest.approx((world - 1) / 2 + 0.5)
    assert red_m["actor/x_max"] == world - 1 and red_m["actor/y_min"] == 0

    # ---------------------------------------------------------------- replica check catches a divergent rank
    if rank == world - 1:
        with torch.no_grad():
            next(a.parameters()).view(-1)[0] += 1.0
    rc = replica_check(a, rep, {}, (), 0.0)
    assert not rc["replicas_identical"] and not rc["weights_equal"], rc
    emu.disable()
    dist.destroy_process_group()


def test_world8_rccl_branches_match_single_process():
    port = _free_port()
    mp.spawn(_worker, args=(WORLD, port), nprocs=WORLD, join=True)
