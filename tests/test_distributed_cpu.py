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
