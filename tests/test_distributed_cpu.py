"""Multi-process (gloo, world size 2) tests of the data-parallel plumbing, on CPU:
bucketed gradient all-reduce, distributed stats (closed forms of the reference's
tests/utils/test_torch_functional.py:25-117), DP_COMPUTE_PROTO dispatch/collect."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)


def _run(fn, world=2):
    port = _free_port()
    mp.spawn(fn, args=(world, port), nprocs=world, join=True)


# ------------------------------------------------------------------ gradient bucket reducer
def _model(seed=0):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(6, 16), torch.nn.Tanh(), torch.nn.Linear(16, 3))


def _reducer_worker(rank, world, port):
    _init(rank, world, port)
    from verl_amd.workers.grad_sync import GradBucketReducer

    model = _model()
    red = GradBucketReducer(model.parameters(), bucket_bytes=256)  # tiny buckets: several of them
    assert len(red.buckets) > 1
    g = torch.Generator().manual_seed(100)
    xs = [torch.randn(4, 6, generator=g) for _ in range(world * 2)]  # 2 micro-batches per rank
    red.zero_grad()
    mine = xs[rank * 2 : rank * 2 + 2]
    for i, x in enumerate(mine):
        if i == len(mine) - 1:
            red.begin_sync()
        (model(x).square().mean() / 2).backward()
    red.finish_sync()
    got = {n: p.grad.clone() for n, p in model.named_parameters()}
    # single-process reference: all micro-batches, loss / (2 * world) each = mean over ranks
    ref = _model()
    for x in xs:
        (ref(x).square().mean() / (2 * world)).backward()
    for n, p in ref.named_parameters():
        assert torch.allclose(got[n], p.grad, atol=1e-6), n
    # second mini-batch: zero_grad keeps the bucket views
    red.zero_grad()
    assert all(p.grad.abs().sum() == 0 for p in model.parameters())
    dist.destroy_process_group()


def test_grad_bucket_reducer_matches_single_process_mean():
    _run(_reducer_worker)


def _mp_worker(rank, world, port):
    _init(rank, world, port)
    from verl_amd.workers.grad_sync import MixedPrecisionParams

    model = _model()
    ref = _model()
    mp_ = MixedPrecisionParams(model, bucket_bytes=256)
    assert all(p.dtype == torch.bfloat16 for p in model.parameters())
    opt = torch.optim.AdamW(mp_.optimizer_params(), lr=1e-2)
    g = torch.Generator().manual_seed(5)
    xs = [torch.randn(4, 6, generator=g) for _ in range(world * 2)]
    mp_.zero_grad()
    for i, x in enumerate(xs[rank * 2 : rank * 2 + 2]):
        if i == 1:
            mp_.begin_sync()
        (model(x.bfloat16()).float().square().mean() / 2).backward()
    mp_.finish_sync()
    # fp32 gradient buckets hold the rank-mean of bf16 gradients (accumulated in fp32)
    refp = {n: p for n, p in ref.named_parameters()}
    bf = _model()
    for p in bf.parameters():
        p.data = p.data.bfloat16()
    for x in xs:
        (bf(x.bfloat16()).float().square().mean() / (2 * world)).backward()
    for (n, p), m in zip(bf.named_parameters(), mp_.optimizer_params(), strict=True):
        assert torch.allclose(m.grad, p.grad.float(), atol=2e-2, rtol=2e-2), n
        assert torch.equal(m.data, refp[n].data)  # masters start as the fp32 init
    opt.step()
    mp_.after_step()
    for p, m in zip(model.parameters(), mp_.optimizer_params(), strict=True):
        assert torch.equal(p.data, m.data.bfloat16())
    flat = torch.cat([m.detach().reshape(-1) for m in mp_.optimizer_params()])
    other = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(other, flat)
    assert torch.equal(other[0], other[1])
    dist.destroy_process_group()


def test_mixed_precision_params_dp():
    _run(_mp_worker)


# ------------------------------------------------------------------ distributed stats
def _stats_worker(rank, world, port):
    _init(rank, world, port)
    from verl_amd.utils.torch_functional import distributed_masked_mean, distributed_mean_max_min_std

    local = torch.tensor([float(rank + 1)])
    mean, gmax, gmin, gstd = distributed_mean_max_min_std(local, True, True, True)
    vals = [float(i + 1) for i in range(world)]
    m = sum(vals) / len(vals)
    assert torch.allclose(mean, torch.tensor(m))
    assert gmax.item() == max(vals) and gmin.item() == min(vals)
    assert torch.allclose(gstd, torch.tensor((sum((v - m) ** 2 for v in vals) / (len(vals) - 1)) ** 0.5))
    t = torch.tensor([rank * 2 + 1.0, rank * 2 + 2.0])
    mask = torch.tensor([1.0, 0.0]) if rank == 0 else torch.tensor([0.0, 1.0])
    gm = distributed_masked_mean(t, mask)
    valid = [1.0] + [2 * i + 2.0 for i in range(1, world)]
    assert torch.allclose(gm, torch.tensor(sum(valid) / len(valid)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_distributed_stats_closed_forms(world):
    port = _free_port()
    mp.spawn(_stats_worker, args=(world, port), nprocs=world, join=True)


# ------------------------------------------------------------------ DP_COMPUTE_PROTO
def _dispatch_worker(rank, world, port):
    _init(rank, world, port)
    from verl_amd.protocol import DataProto, all_gather_data_proto
    from verl_amd.workers.dp_workers import collect_dp_compute_data_proto, dispatch_dp_compute_data_proto

    full = DataProto.from_dict(tensors={"x": torch.arange(8).float()},
                               non_tensors={"uid": np.array([f"u{i // 2}" for i in range(8)], dtype=object)})
    shards = dispatch_dp_compute_data_proto(full, world)
    mine = shards[rank]
    assert mine.batch["x"].tolist() == list(range(rank * 4, rank * 4 + 4))
    out = collect_dp_compute_data_proto(shards)
    assert torch.equal(out.batch["x"], full.batch["x"])
    all_gather_data_proto(mine, None)
    assert torch.equal(mine.batch["x"], full.batch["x"])
    assert list(mine.non_tensor_batch["uid"]) == list(full.non_tensor_batch["uid"])
    dist.destroy_process_group()


def test_dp_dispatch_collect_and_all_gather():
    _run(_dispatch_worker)


# ------------------------------------------------------------------ ordered buckets + rank-0 sync
def _order_worker(rank, world, port):
    _init(rank, world, port)
    from verl_amd.workers.grad_sync import GradBucketReducer

    torch.manual_seed(100 + rank)  # different init per rank: the reducer must sync from rank 0
    model = torch.nn.Sequential(torch.nn.Linear(6, 16), torch.nn.Tanh(), torch.nn.Linear(16, 3))
    red = GradBucketReducer(model.parameters(), bucket_bytes=256)
    flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    parts = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(parts, flat)
    assert all(torch.equal(parts[0], p) for p in parts)
    # launches happen in bucket order even when a later bucket completes first
    launched = []
    orig = red._collective
    red._collective = lambda b: (launched.append(b.index), orig(b))[1]
    red.zero_grad()
    red.begin_sync()
    red._mark_ready(red.buckets[-1])  # last bucket ready first: nothing may launch yet
    assert launched == []
    for b in red.buckets[:-1]:
        red._mark_ready(b)
    red.finish_sync()
    assert launched == list(range(len(red.buckets)))
    dist.destroy_process_group()


def test_reducer_syncs_rank0_params_and_orders_collectives():
    _run(_order_worker)


# ------------------------------------------------------------------ ZeRO-sharded masters
def _zero_worker(rank, world, port):
    _init(rank, world, port)
    from verl_amd.workers.grad_sync import MixedPrecisionParams, ShardedMixedPrecisionParams

    def model():
        torch.manual_seed(0)
        return torch.nn.Sequential(torch.nn.Linear(6, 40), torch.nn.Tanh(), torch.nn.Linear(40, 3))

    a, b = model(), model()
    rep = MixedPrecisionParams(a, bucket_bytes=512)
    shd = ShardedMixedPrecisionParams(b, bucket_bytes=512)
    assert len(shd.buckets) > 1
    opt_a = torch.optim.AdamW(rep.optimizer_params(), lr=1e-2, weight_decay=0.01, foreach=False)
    opt_b = torch.optim.AdamW(shd.optimizer_params(), lr=1e-2, weight_decay=0.01, foreach=False)
    g = torch.Generator().manual_seed(5)
    xs = [torch.randn(4, 6, generator=g) for _ in range(world * 2)]
    for step in range(3):
        for mgr, mod, opt in ((rep, a, opt_a), (shd, b, opt_b)):
            mgr.zero_grad()
            for i, x in enumerate(xs[rank * 2 : rank * 2 + 2]):
                if i == 1:
                    mgr.begin_sync()
                (mod(x.bfloat16() + step).float().square().mean() / 2).backward()
            mgr.finish_sync()
        n_rep = torch.nn.utils.clip_grad_norm_(rep.optimizer_params(), max_norm=0.5, foreach=True)
        n_shd = shd.clip_grad_norm_(0.5)
        assert torch.allclose(n_rep, n_shd, rtol=1e-5), (n_rep, n_shd)
        opt_a.step()
        opt_b.step()
        rep.after_step()
        shd.after_step()
        for (n, p), q in zip(a.named_parameters(), b.parameters(), strict=True):
            assert p.dtype == q.dtype == torch.bfloat16
            assert torch.allclose(p.float(), q.float(), atol=1e-2, rtol=0), (step, n)
        # the shards of the masters equal the replicated masters (fp32)
        full = torch.cat([m.detach().reshape(-1) for m in reversed(rep.optimizer_params())])
        mine = torch.cat([s.detach() for s in shd.shards])
        per = [s.numel() for s in shd.shards]
        offs, o = [], 0
        for bkt, n_per in zip(shd.buckets, per, strict=True):
            n_real = sum(p.numel() for p in bkt.params)
            lo = rank * n_per
            hi = min(lo + n_per, n_real)
            if hi > lo:
                got = shd.shards[bkt.index].detach()[: hi - lo]
                want = full[o + lo : o + hi]
                assert torch.allclose(got, want, atol=1e-6, rtol=1e-5), (step, bkt.index)
            o += n_real
        del mine, offs
    mem = shd.memory_bytes()
    assert mem["fp32_master_shard"] * world >= sum(p.numel() for p in b.parameters()) * 4
    dist.destroy_process_group()


def test_zero_sharded_masters_match_replicated_dp():
    _run(_zero_worker)


# ------------------------------------------------------------------ cross-rank group scores
def _gather_worker(rank, world, port):
    _init(rank, world, port)
    from verl_amd.trainer.ppo.dp_algos import check_groups_intact, gather_row_scores, uid_keys

    # rank r holds rows [3r, 3r + 3) of a 3W-row batch whose groups straddle the ranks
    rows = list(range(3 * rank, 3 * rank + 3))
    uids = np.array([f"g{i // 2}" for i in rows], dtype=object)
    scores = torch.tensor([float(i) for i in rows])
    lens = torch.tensor([10.0 + i for i in rows])
    s_all, l_all, keys, off = gather_row_scores(scores, lens, uids, None)
    assert off == 3 * rank
    assert s_all.tolist() == [float(i) for i in range(3 * world)]
    assert l_all.tolist() == [10.0 + i for i in range(3 * world)]
    full_uids = np.array([f"g{i // 2}" for i in range(3 * world)], dtype=object)
    assert (keys == uid_keys(full_uids)).all()
    assert not check_groups_intact(uids)
    assert check_groups_intact(np.array([f"r{rank}-{i}" for i in range(3)], dtype=object))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_row_scores_rank_order(world):
    port = _free_port()
    mp.spawn(_gather_worker, args=(world, port), nprocs=world, join=True)


def test_uid_keys_distinguish_types_and_values():
    from verl_amd.trainer.ppo.dp_algos import uid_keys

    k = uid_keys(np.array(["a", "b", "a", 1, "1"], dtype=object))
    assert k[0] == k[2] and k[0] != k[1] and k[3] != k[4]
    assert (k >= 0).all()


@pytest.mark.parametrize("zero", [False, True])
def test_dropped_worker_frees_its_parameters(zero):
    """The gradient hooks the parameter managers put on the parameters hold them only weakly: a
    worker that is dropped releases its model, masters, gradient buckets and optimizer state (a
    bound-method hook kept all of it alive for the process lifetime — 130+ GB per 7-8B worker)."""
    import gc
    import weakref

    from verl_amd.utils.config import AttrDict, actor_config
    from verl_amd.utils.model import build_qwen2
    from verl_amd.workers.dp_workers import ActorWorker

    m = build_qwen2("tiny", device="cpu", seed=0, attn_implementation="sdpa")
    w = ActorWorker(AttrDict(actor=actor_config(ppo_mini_batch_size=4, ppo_micro_batch_size_per_gpu=2),
                             rollout=AttrDict(n=1, temperature=1.0, log_prob_micro_batch_size_per_gpu=2)), rollout_n=1)
    w.init_model(m, zero=zero)
    refs = [weakref.ref(p) for p in m.parameters()] + [weakref.ref(w.actor.grad_reducer)]
    del m, w
    gc.collect()
    assert all(r() is None for r in refs)


@pytest.mark.parametrize("max_norm", [1e-3, 1e3])
def test_bucket_clip_equals_torch_clip(max_norm):
    """MixedPrecisionParams.clip_grad_norm_ (flat fp32 buckets) = torch.nn.utils.clip_grad_norm_ on
    the masters: same norm, same clipped gradients (to fp32 reduction-order rounding)."""
    from verl_amd.workers.grad_sync import MixedPrecisionParams

    def model():
        torch.manual_seed(0)
        return torch.nn.Sequential(torch.nn.Linear(6, 16), torch.nn.Tanh(), torch.nn.Linear(16, 3))

    a, b = model(), model()
    ma, mb = MixedPrecisionParams(a, bucket_bytes=256), MixedPrecisionParams(b, bucket_bytes=256)
    assert len(ma.buckets) > 1
    x = torch.randn(5, 6, generator=torch.Generator().manual_seed(1))
    for mod, mgr in ((a, ma), (b, mb)):
        mod(x.bfloat16()).float().square().sum().backward()
        mgr.finish_sync()
    n_torch = torch.nn.utils.clip_grad_norm_(ma.optimizer_params(), max_norm=max_norm, foreach=True)
    n_mine = mb.clip_grad_norm_(max_norm)
    assert torch.allclose(n_torch, n_mine, rtol=1e-6), (n_torch, n_mine)
    for p, q in zip(ma.optimizer_params(), mb.optimizer_params(), strict=True):
        assert torch.allclose(p.grad, q.grad, rtol=1e-6, atol=1e-9)


# ------------------------------------------------------------------ batch-global agg_loss metric
def _agg_dp_worker(rank, world, port):
    _init(rank, world, port)
    from oracle import reference_ops as ref
    from verl_amd.trainer.ppo.dp_algos import agg_loss_dp

    g = torch.Generator().manual_seed(7)
    B, R = 6, 9
    x = torch.randn(world * B, R, generator=g)
    mask = (torch.rand(world * B, R, generator=g) > 0.3).long()
    mask[:, 0] = 1
    mask[1, 3:] = 0  # unequal token counts per row and per rank
    mine = slice(rank * B, (rank + 1) * B)
    for mode in ("token-mean", "seq-mean-token-sum", "seq-mean-token-mean", "seq-mean-token-sum-norm"):
        got = agg_loss_dp(x[mine], mask[mine], mode)
        want = ref.agg_loss(x, mask, mode)  # the reference's driver: agg_loss over the whole batch
        assert torch.allclose(got, want.float(), rtol=1e-6, atol=1e-6), (mode, float(got), float(want))
    with pytest.raises(ValueError, match="Invalid loss_agg_mode"):
        agg_loss_dp(x[mine], mask[mine], "bogus")
    dist.destroy_process_group()


def test_agg_loss_dp_equals_whole_batch_agg_loss():
    """the actor/entropy metric is agg_loss over the WHOLE batch on the reference's
    driver (ray_trainer.py:1224-1228); each rank's shard reduces to (numerator, denominator) and one
    all-reduce gives the same value for every agg mode."""
    _run(_agg_dp_worker)
