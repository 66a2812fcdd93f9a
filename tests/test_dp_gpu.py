"""Data-parallel correctness on one MI355X: two ranks (gloo process group, both on cuda:0) must
reproduce the single-process results — global GAE whitening, masked whitening, and one full
actor update (bucketed gradient all-reduce + AdamW)."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _gae_worker(rank, world, port):
    _init(rank, world, port)
    from verl_amd import kernels as K
    from verl_amd.trainer.ppo.dp_algos import compute_gae_advantage_return_dp, masked_whiten_dp

    g = torch.Generator().manual_seed(0)
    B, R = 24, 300
    rewards = torch.randn(B, R, generator=g) * (torch.rand(B, R, generator=g) > 0.9)
    values = torch.randn(B, R, generator=g)
    lens = torch.randint(1, R + 1, (B,), generator=g)
    mask = (torch.arange(R)[None, :] < lens[:, None]).long()
    full_adv, full_ret = K.gae_advantage_return(rewards.cuda(), values.cuda(), mask.cuda(), 0.99, 0.95)
    sl = slice(rank * B // world, (rank + 1) * B // world)
    adv, ret = compute_gae_advantage_return_dp(rewards[sl].cuda(), values[sl].cuda(), mask[sl].cuda(), 0.99, 0.95)
    assert torch.equal(ret, full_ret[sl])
    assert torch.allclose(adv, full_adv[sl], atol=2e-6, rtol=1e-6), (adv - full_adv[sl]).abs().max()
    x = torch.randn(B, R, generator=g).cuda()
    stats, _ = K.whiten_stats(x, mask.cuda())
    want = K.whiten_apply(x, mask.cuda(), stats)
    got = masked_whiten_dp(x[sl], mask[sl].cuda())
    assert torch.allclose(got, want[sl], atol=2e-6, rtol=1e-6)
    dist.destroy_process_group()


def test_gae_and_whiten_dp_equal_single_process():
    mp.spawn(_gae_worker, args=(2, _free_port()), nprocs=2, join=True)


def _update_worker(rank, world, port):
    _init(rank, world, port)
    from verl_amd.utils.config import actor_config
    from verl_amd.utils.model import build_qwen2
    from verl_amd.utils.synthetic import make_grpo_batch
    from verl_amd.workers.actor import DataParallelPPOActor
    from verl_amd.workers.grad_sync import GradBucketReducer

    dev = torch.device("cuda", 0)
    data = make_grpo_batch(n_prompts=2, n=4, prompt_len=16, response_len=24, vocab=4096, min_prompt=3,
                           dense_responses=False, min_response=4, seed=7, device=dev)
    b = data.batch
    g = torch.Generator(device=dev).manual_seed(3)
    b["old_log_probs"] = -torch.rand(b["responses"].shape, device=dev, generator=g)
    b["advantages"] = torch.randn(b["responses"].shape, device=dev, generator=g) * b["response_mask"]
    b["ref_log_prob"] = b["old_log_probs"] + 0.1
    data.meta_info["temperature"] = 1.0

    def make(reduced):
        model = build_qwen2("tiny", device=dev, attn_implementation="sdpa", seed=11)
        cfg = actor_config(use_remove_padding=False, autocast_dtype=None, ppo_micro_batch_size_per_gpu=2,
                           ppo_mini_batch_size=8 // (world if reduced else 1), use_kl_loss=True, grad_clip=1e9)
        opt = torch.optim.AdamW(model.parameters(), lr=1e-3)
        red = GradBucketReducer(model.parameters(), bucket_bytes=1 << 16) if reduced else None
        return model, DataParallelPPOActor(cfg, model, opt, grad_reducer=red)

    model, actor = make(True)
    shard = data[rank * 4 : (rank + 1) * 4]
    actor.update_policy(shard)
    if rank == 0:
        ref_model, ref_actor = make(False)
        ref_actor.update_policy(data)
        for (n, p), (_, q) in zip(model.named_parameters(), ref_model.named_parameters(), strict=True):
            assert torch.allclose(p, q, atol=1e-6, rtol=1e-5), (n, (p - q).abs().max().item())
    # both ranks hold identical parameters after the step
    flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).cpu()
    other = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(other, flat)
    assert torch.equal(other[0], other[1])
    dist.destroy_process_group()


def test_actor_update_dp2_equals_single_process():
    mp.spawn(_update_worker, args=(2, _free_port()), nprocs=2, join=True)
