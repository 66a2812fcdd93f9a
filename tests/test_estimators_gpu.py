"""Remaining advantage estimators and policy-loss variants on MI355X against
the oracle restatements: pass@k and OPO (group-kernel epilogues), REINFORCE++ and ReMax (chunked
reverse-scan kernel), GPG, and the gpg / clip_cov / kl_cov policy losses."""

import numpy as np
import pytest
import torch

from oracle import reference_ops as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(a, b, atol=1e-5, rtol=1e-5, what=""):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    assert a.shape == b.shape, (what, a.shape, b.shape)
    err = (a - b).abs()
    assert bool((err <= atol + rtol * b.abs()).all()), f"{what}: max err {err.max().item():.3e}"


def _outcome_batch(G=6, n=5, R=33, seed=0, ties=False, singletons=False):
    g = torch.Generator().manual_seed(seed)
    B = G * n
    rew = torch.zeros(B, R)
    lens = torch.randint(1, R + 1, (B,), generator=g)
    mask = (torch.arange(R)[None, :] < lens[:, None]).to(torch.int64)
    sc = torch.randint(0, 3, (B,), generator=g).float() if ties else torch.randn(B, generator=g)
    rew[torch.arange(B), lens - 1] = sc
    rew += 0.01 * torch.randn(B, R, generator=g) * (0 if ties else 1)  # unmasked-sum semantics
    uids = np.array([f"p{i % G}" for i in range(B)], dtype=object)  # interleaved groups
    if singletons:
        uids[0] = "solo_a"
        uids[-1] = "solo_b"
    return rew, mask, uids


def _cfg(**kw):
    from verl_amd.utils.config import AttrDict

    return AttrDict(**kw)


@pytest.mark.parametrize("norm", [True, False])
@pytest.mark.parametrize("ties", [False, True])
def test_grpo_passk(norm, ties):
    from verl_amd.trainer.ppo import core_algos

    rew, mask, uids = _outcome_batch(seed=1, ties=ties)
    want, _ = ref.compute_grpo_passk_outcome_advantage(rew.clone(), mask, uids, norm=norm)
    got, _ = core_algos.compute_grpo_passk_outcome_advantage(rew.to(DEV), mask.to(DEV), uids,
                                                            config=_cfg(norm_adv_by_std_in_grpo=norm))
    _close(got, want, what="passk")
    uids2 = uids.copy()
    uids2[3] = "lonely"
    with pytest.raises(ValueError, match="Pass@k requires at least 2 samples per group"):
        core_algos.compute_grpo_passk_outcome_advantage(rew.to(DEV), mask.to(DEV), uids2, config=_cfg())


@pytest.mark.parametrize("mask_dtype", [torch.int64, torch.float32])
def test_opo(mask_dtype):
    from verl_amd.trainer.ppo import core_algos

    rew, mask, uids = _outcome_batch(seed=2, singletons=True)
    mask = mask.to(mask_dtype)
    want, _ = ref.compute_opo_outcome_advantage(rew.clone(), mask, uids)
    got, _ = core_algos.compute_opo_outcome_advantage(rew.to(DEV), mask.to(DEV), uids)
    _close(got, want, what="opo")


@pytest.mark.parametrize("R", [1, 17, 64, 1024, 3000])
@pytest.mark.parametrize("gamma", [1.0, 0.99])
def test_reinforce_plus_plus(R, gamma):
    from verl_amd.trainer.ppo import core_algos

    g = torch.Generator().manual_seed(R)
    B = 13
    rew = torch.randn(B, R, generator=g)
    lens = torch.randint(1, R + 1, (B,), generator=g)
    mask = (torch.arange(R)[None, :] < lens[:, None]).to(torch.int64)
    mask[0, : R // 2] = 0  # multi-turn style holes: the return resets across them
    mask[0, R // 2 :] = 1
    if mask.sum() < 2:
        mask[1, :] = 1
    want_adv, want_ret = ref.compute_reinforce_plus_plus_outcome_advantage(rew.double(), mask, gamma)
    got_adv, got_ret = core_algos.compute_reinforce_plus_plus_outcome_advantage(rew.to(DEV), mask.to(DEV),
                                                                               config=_cfg(gamma=gamma))
    # chunked scan reassociates the recurrence: budget against the float64 twin (as for GAE)
    tol = 1e-4 * max(1.0, (R ** 0.5) / 8)
    _close(got_ret, want_ret, atol=tol, rtol=tol, what="rf++ returns")
    _close(got_adv, want_adv, atol=tol, rtol=tol, what="rf++ advantages")


@pytest.mark.parametrize("R", [5, 1024])
def test_remax(R):
    from verl_amd.trainer.ppo import core_algos

    g = torch.Generator().manual_seed(3)
    B = 9
    rew = torch.randn(B, R, generator=g)
    lens = torch.randint(1, R + 1, (B,), generator=g)
    mask = (torch.arange(R)[None, :] < lens[:, None]).to(torch.int64)
    base = torch.randn(B, generator=g)
    want_adv, want_ret = ref.compute_remax_outcome_advantage(rew.double(), base.double(), mask)
    got_adv, got_ret = core_algos.compute_remax_outcome_advantage(rew.to(DEV), base.to(DEV), mask.to(DEV))
    tol = 1e-4 * max(1.0, (R ** 0.5) / 8)
    _close(got_ret, want_ret, atol=tol, rtol=tol, what="remax returns")
    _close(got_adv, want_adv, atol=tol, rtol=tol, what="remax advantages")


def test_gpg_advantage():
    from verl_amd.trainer.ppo import core_algos

    rew, mask, uids = _outcome_batch(seed=4, singletons=True, ties=True)
    want, _ = ref.compute_gpg_outcome_advantage(rew.clone(), mask, uids, f_norm=2.0)
    got, _ = core_algos.compute_gpg_outcome_advantage(rew.to(DEV), mask.to(DEV), uids, f_norm=2.0)
    _close(got, want, what="gpg")


def _policy_inputs(B=6, R=200, seed=0):
    g = torch.Generator().manual_seed(seed)
    old = -torch.rand(B, R, generator=g) * 3
    lp = old + 0.3 * torch.randn(B, R, generator=g)
    adv = torch.randn(B, R, generator=g)
    lens = torch.randint(1, R + 1, (B,), generator=g)
    mask = (torch.arange(R)[None, :] < lens[:, None]).to(torch.int64)
    return old, lp, adv, mask


def _actor_cfg():
    from verl_amd.utils.config import actor_config

    return actor_config()


@pytest.mark.parametrize("agg", ["token-mean", "seq-mean-token-mean"])
def test_gpg_loss(agg):
    from verl_amd.trainer.ppo import core_algos

    old, lp, adv, mask = _policy_inputs(seed=5)
    a = lp.clone().requires_grad_(True)
    want = ref.compute_policy_loss_gpg(a, adv, mask, agg)
    want.backward()
    b = lp.to(DEV).requires_grad_(True)
    fn = core_algos.get_policy_loss_fn("gpg")
    got = fn(old.to(DEV), b, adv.to(DEV), mask.to(DEV), agg, _actor_cfg())[0]
    got.backward()
    _close(got, want, what="gpg loss")
    _close(b.grad, a.grad, atol=1e-7, what="gpg grad")


def test_kl_cov_loss():
    from verl_amd.trainer.ppo import core_algos

    old, lp, adv, mask = _policy_inputs(B=8, R=900, seed=6)
    cfg = _actor_cfg()
    cfg.policy_loss.kl_cov_ratio = 0.01
    a = lp.clone().requires_grad_(True)
    want, want_kl = ref.compute_policy_loss_kl_cov(old, a, adv, mask, kl_cov_ratio=0.01, ppo_kl_coef=0.1)
    want.backward()
    b = lp.to(DEV).requires_grad_(True)
    got, _, got_kl, _ = core_algos.get_policy_loss_fn("kl_cov")(old.to(DEV), b, adv.to(DEV), mask.to(DEV),
                                                                "token-mean", cfg)
    got.backward()
    _close(got, want, what="kl_cov loss")
    _close(got_kl, want_kl, what="kl_cov ppo_kl")
    _close(b.grad, a.grad, atol=1e-7, what="kl_cov grad")


def test_clip_cov_loss_same_seed_same_selection():
    """clip_cov draws a random subset (torch.randperm on the default CPU generator, as the
    reference): with the same seed the selection, loss and gradient match."""
    from verl_amd.trainer.ppo import core_algos

    old, lp, adv, mask = _policy_inputs(B=8, R=900, seed=7)
    cfg = _actor_cfg()
    cfg.policy_loss.clip_cov_ratio = 0.02
    cfg.policy_loss.clip_cov_lb = 0.0
    cfg.policy_loss.clip_cov_ub = 5.0
    a = lp.clone().requires_grad_(True)
    torch.manual_seed(123)
    b = lp.to(DEV).requires_grad_(True)
    got = core_algos.get_policy_loss_fn("clip_cov")(old.to(DEV), b, adv.to(DEV), mask.to(DEV), "token-mean", cfg)
    got[0].backward()
    # CPU restatement of the same reference lines, same seed
    torch.manual_seed(123)
    neg = a - old
    ratio = torch.exp(neg)
    l1 = -adv * ratio
    l2 = -adv * torch.clamp(ratio, 1 - 0.2, 1 + 0.2)
    clip_by_origin = (l2 > l1) & (mask > 0)
    cov = (adv - ref.masked_mean(adv, mask)) * (a - ref.masked_mean(a.detach(), mask))
    cov[mask == 0] = -torch.inf
    cov[clip_by_origin] = -torch.inf
    num = max(int(0.02 * mask.sum().item()), 1)
    idx = torch.nonzero((cov < 5.0) & (cov > 0.0) & (mask > 0))
    idx = idx[torch.randperm(len(idx))[: min(num, len(idx))]]
    corr = torch.ones_like(adv)
    corr[idx[:, 0], idx[:, 1]] = 0
    loss = ref.agg_loss(torch.maximum(l1, l2) * corr, mask, "token-mean")
    loss.backward()
    _close(got[0], loss, what="clip_cov loss")
    _close(got[1], ref.masked_mean((corr == 0).float(), mask), what="clip_cov clipfrac")
    _close(b.grad, a.grad, atol=1e-7, what="clip_cov grad")


@pytest.mark.parametrize("agg", ["token-mean", "seq-mean-token-sum", "seq-mean-token-mean", "seq-mean-token-sum-norm"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_compute_entropy_loss_matches_oracle(agg, dtype):
    """a9, core_algos.py:975-989: agg_loss(entropy_from_logits(logits)) over [bs, R, V] logits, value
    and gradient w.r.t. the logits (the entropy-regularisation term's backward through the fused
    entropy kernel and the masked aggregation) against the oracle's eager restatement in fp32."""
    from verl_amd.trainer.ppo import core_algos

    g = torch.Generator().manual_seed(7)
    bs, R, V = 5, 37, 1000
    logits = (2.0 * torch.randn(bs, R, V, generator=g)).to(dtype)
    lens = torch.randint(1, R + 1, (bs,), generator=g)
    mask = (torch.arange(R)[None, :] < lens[:, None]).to(torch.int64)
    x = logits.to(DEV).requires_grad_(True)
    got = core_algos.compute_entropy_loss(x, mask.to(DEV), loss_agg_mode=agg)
    got.backward()
    xr = logits.float().requires_grad_(True)
    want = ref.agg_loss(ref.entropy_from_logits(xr), mask.float(), agg)
    want.backward()
    _close(got, want, atol=1e-5, rtol=1e-5, what=f"entropy loss {agg}")
    tol = 1e-6 if dtype == torch.float32 else 4e-3  # bf16 logits: gradient rounded to bf16
    _close(x.grad.float(), xr.grad, atol=tol, rtol=1e-2 if dtype != torch.float32 else 1e-4,
           what=f"entropy loss grad {agg}")
