"""Cross-rank group statistics on one MI355X (2 ranks, gloo, both on cuda:0): a 512 x 1024 GRPO
batch is Karmarkar-Karp balanced over the ranks (which splits prompt groups, as the reference's
_balance_batch does before compute_advantage, ray_trainer.py:1204-1205, 262-273), chunked as
DP_COMPUTE_PROTO does, and every rank's advantages must equal the single-process oracle over the
whole batch (1e-5) for the group estimators, and the whitened ones (GAE, RF++, RF++-baseline)."""

import os
import socket

import numpy as np
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


def _batch(seed=1234, continuous=True):
    from verl_amd.utils.synthetic import make_grpo_batch

    data = make_grpo_batch(64, 8, 256, 1024, vocab=1000, dense_responses=False, seed=seed)
    if continuous:  # distinct scores: pass@k's argmax has no ties
        g = torch.Generator().manual_seed(seed + 1)
        r = data.batch["token_level_rewards"]
        last = data.batch["response_mask"].sum(-1) - 1
        r.zero_()
        r[torch.arange(r.shape[0]), last] = torch.randn(r.shape[0], generator=g)
        r += 0.01 * torch.randn(r.shape, generator=g) * data.batch["response_mask"]
    data.batch["values"] = torch.randn(data.batch["token_level_rewards"].shape,
                                       generator=torch.Generator().manual_seed(seed + 2))
    return data


def _worker(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import reference_ops as ref
    from verl_amd.trainer.ppo.core_algos import AdvantageEstimator
    from verl_amd.trainer.ppo.dp_algos import check_groups_intact, compute_advantage_dp
    from verl_amd.trainer.ppo.ray_trainer import balance_batch
    from verl_amd.utils.config import AttrDict

    for continuous in (True, False):
        full = _batch(continuous=continuous)
        balance_batch(full, world, {})
        shard = full.chunk(world)[rank]
        assert not check_groups_intact(shard.non_tensor_batch["uid"])  # groups really are split
        sl = slice(rank * len(shard), (rank + 1) * len(shard))
        rw = full.batch["token_level_rewards"]
        m = full.batch["response_mask"]
        idx = full.non_tensor_batch["uid"]
        cases = [
            (AdvantageEstimator.GRPO, dict(norm_adv_by_std_in_grpo=True),
             ref.compute_grpo_outcome_advantage(rw.clone(), m, idx)[0]),
            (AdvantageEstimator.GRPO, dict(norm_adv_by_std_in_grpo=False),
             ref.compute_grpo_outcome_advantage(rw.clone(), m, idx, norm_adv_by_std_in_grpo=False)[0]),
            (AdvantageEstimator.RLOO, {}, ref.compute_rloo_outcome_advantage(rw.clone(), m, idx)[0]),
            (AdvantageEstimator.OPO, {}, ref.compute_opo_outcome_advantage(rw.clone(), m, idx)[0]),
            (AdvantageEstimator.GPG, {}, ref.compute_gpg_outcome_advantage(rw.clone(), m, idx)[0]),
            (AdvantageEstimator.REINFORCE_PLUS_PLUS_BASELINE, {},
             ref.compute_reinforce_plus_plus_baseline_outcome_advantage(rw.clone(), m, idx)[0]),
            (AdvantageEstimator.REINFORCE_PLUS_PLUS, dict(config=AttrDict(gamma=0.99)),
             ref.compute_reinforce_plus_plus_outcome_advantage(rw.clone(), m, 0.99)[0]),
            (AdvantageEstimator.GAE, dict(gamma=0.99, lam=0.95),
             ref.compute_gae_advantage_return(rw.clone(), full.batch["values"], m, 0.99, 0.95)[0]),
        ]
        if continuous:
            cases.append((AdvantageEstimator.GRPO_PASSK, dict(config=AttrDict(norm_adv_by_std_in_grpo=True)),
                          ref.compute_grpo_passk_outcome_advantage(rw.clone(), m, idx)[0]))
        for est, kw, want in cases:
            d = shard.to(torch.device("cuda", 0))
            compute_advantage_dp(d, est, **kw)
            got = d.batch["advantages"].cpu()
            tol = 1e-4 if est == AdvantageEstimator.GAE else 1e-5
            assert torch.allclose(got, want[sl], atol=tol, rtol=tol), (est, kw, (got - want[sl]).abs().max().item())
    dist.destroy_process_group()


def test_group_advantages_dp2_with_split_groups_equal_single_process_oracle():
    mp.spawn(_worker, args=(2, _free_port()), nprocs=2, join=True)


def test_outcome_three_phase_kernels_equal_oracle_at_16x():
    """Single process at 16x the headline (8,192 x 1,024): the three-phase outcome kernels
    (row scores -> group coefficients -> broadcast) against the oracle."""
    from oracle import reference_ops as ref
    from verl_amd import _lib as L
    from verl_amd import kernels as K

    g = torch.Generator().manual_seed(0)
    B, R, n = 8192, 1024, 8
    rw = torch.zeros(B, R)
    lens = torch.randint(1, R + 1, (B,), generator=g)
    rw[torch.arange(B), lens - 1] = torch.randn(B, generator=g)
    mask = (torch.arange(R)[None, :] < lens[:, None]).long()
    idx = np.array([f"p{i}" for i in np.random.RandomState(0).permutation(B) // n], dtype=object)
    want = ref.compute_grpo_outcome_advantage(rw.clone(), mask, idx)[0]
    got = K.outcome_advantage(rw.cuda(), mask.cuda(), idx, 1e-6, L.VA_ADV_GRPO).cpu()
    assert torch.allclose(got, want, atol=1e-5, rtol=1e-5)
