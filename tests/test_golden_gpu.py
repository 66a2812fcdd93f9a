"""GPU kernels vs the committed golden fixtures (tests/golden/golden_config1.npz, BASELINE config 1),
and headline-size (512 x 1024, V = 151,936) parity: the full core-algos batch against the oracle,
the log-prob kernel on sampled rows of a full micro-batch plus size-independent invariants."""

import os

import numpy as np
import pytest
import torch

from oracle import reference_ops as ref
from tests.golden.make_golden import LOGIT_CASES, logits_case

pytestmark = pytest.mark.gpu
DEV = "cuda"
G = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden_config1.npz"), allow_pickle=False)


def t(name, dtype=None):
    x = torch.from_numpy(G[name])
    return (x if dtype is None else x.to(dtype)).to(DEV)


def close(a, b, atol, rtol, what):
    a = a.detach().double().cpu().numpy()
    b = np.asarray(b, dtype=np.float64)
    assert np.allclose(a, b, atol=atol, rtol=rtol, equal_nan=True), f"{what}: max err {np.nanmax(np.abs(a - b)):.3e}"


def test_golden_grpo_and_gae():
    from verl_amd.trainer.ppo import core_algos

    uid = G["uid"]
    adv, ret = core_algos.compute_grpo_outcome_advantage(t("rewards"), t("mask"), uid)
    close(adv, G["grpo_adv"], 1e-5, 1e-5, "grpo")
    assert torch.equal(adv, ret)
    adv, _ = core_algos.compute_grpo_outcome_advantage(t("rewards"), t("mask"), uid, norm_adv_by_std_in_grpo=False)
    close(adv, G["grpo_nostd_adv"], 1e-6, 1e-6, "dr.grpo")
    for tag, (g, lam) in {"g1": (1.0, 1.0), "g099": (0.99, 0.95)}.items():
        a, r = core_algos.compute_gae_advantage_return(t("rewards"), t("values"), t("mask"), g, lam)
        close(r, G[f"gae_{tag}_ret"], 1e-4, 1e-4, f"gae {tag} returns")
        close(a, G[f"gae_{tag}_adv"], 1e-4, 1e-4, f"gae {tag} advantages")


@pytest.mark.parametrize("agg", ["token-mean", "seq-mean-token-sum", "seq-mean-token-mean", "seq-mean-token-sum-norm"])
def test_golden_policy_loss(agg):
    from verl_amd import kernels as K

    lp = t("new").requires_grad_(True)
    out = K.fused_policy_loss(t("old"), lp, t("grpo_adv"), t("mask"), 0.2, 0.28, 3.0, agg, ref_log_prob=t("ref"),
                              kl_loss_type="low_var_kl")
    (out[0] + 0.001 * out[4]).backward()
    key = agg.replace("-", "_")
    want = G[f"loss_{key}_scalars"]
    close(out[[0, 1, 2, 3, 4]], want, 1e-5, 1e-4, f"{agg} scalars")
    g = G[f"loss_{key}_dlp"]
    close(lp.grad, g, 1e-6 * np.abs(g).max() + 1e-12, 1e-4, f"{agg} dlp")


def test_golden_kl():
    from verl_amd.trainer.ppo import core_algos

    for kt in ["kl", "abs", "mse", "low_var_kl"]:
        close(core_algos.kl_penalty(t("new"), t("ref"), kt), G[f"kl_{kt}"], 1e-6, 1e-5, kt)


@pytest.mark.parametrize("case", LOGIT_CASES, ids=[c[0] for c in LOGIT_CASES])
def test_golden_logprob(case):
    from verl_amd.utils import torch_functional as vF

    name, seed, rows, V, dt, T = case
    logits, labels = logits_case(seed, rows, V)
    logits = logits.to(getattr(torch, dt)).to(DEV)
    assert np.array_equal(labels.numpy(), G[f"lp_{name}_labels"])
    lp, ent = vF.logprobs_and_entropy_from_logits(logits, labels.to(DEV), T)
    close(lp, G[f"lp_{name}_logp"], 1e-4, 1e-4, f"{name} logp")
    close(ent, G[f"lp_{name}_entropy"], 1e-4, 1e-4, f"{name} entropy")


# ------------------------------------------------------------------ headline sizes
def test_headline_core_algos_512x1024():
    """GRPO, GAE and the fused loss at the headline batch against the oracle (full batch)."""
    from verl_amd import kernels as K
    from verl_amd.trainer.ppo import core_algos

    g = torch.Generator().manual_seed(42)
    B, R = 512, 1024
    lens = torch.randint(128, R + 1, (B,), generator=g)
    mask = (torch.arange(R)[None, :] < lens[:, None]).long()
    rewards = torch.zeros(B, R)
    rewards[torch.arange(B), lens - 1] = torch.bernoulli(torch.full((B,), 0.5), generator=g)
    uid = np.array([f"p{i // 8}" for i in range(B)], dtype=object)[torch.randperm(B, generator=g).numpy()]
    want, _ = ref.compute_grpo_outcome_advantage(rewards.clone(), mask, uid)
    got, _ = core_algos.compute_grpo_outcome_advantage(rewards.to(DEV), mask.to(DEV), uid)
    close(got, want.numpy(), 1e-5, 1e-5, "grpo 512x1024")
    values = torch.randn(B, R, generator=g)
    wa, wr = ref.compute_gae_advantage_return(rewards.double(), values.double(), mask.double(), 1.0, 1.0)
    a, r = core_algos.compute_gae_advantage_return(rewards.to(DEV), values.to(DEV), mask.to(DEV), 1.0, 1.0)
    close(r, wr.numpy(), 4e-4, 1e-4, "gae returns 512x1024 (vs fp64 twin)")
    close(a, wa.numpy(), 4e-4, 1e-4, "gae adv 512x1024 (vs fp64 twin)")
    new = -torch.rand(B, R, generator=g) * 3
    old = new + 0.05 * torch.randn(B, R, generator=g)
    refl = new + 0.1 * torch.randn(B, R, generator=g)
    newr = new.clone().requires_grad_(True)
    loss, met = ref.actor_loss(old, newr, want, mask, ref_log_prob=refl, kl_loss_type="low_var_kl")
    loss.backward()
    nd = new.to(DEV).requires_grad_(True)
    out = K.fused_policy_loss(old.to(DEV), nd, got, mask.to(DEV), 0.2, 0.2, 3.0, "token-mean", ref_log_prob=refl.to(DEV),
                              kl_loss_type="low_var_kl")
    (out[0] + 0.001 * out[4]).backward()
    close(out[0], met["pg_loss"].item(), 1e-5, 1e-4, "pg_loss")
    close(out[4], met["kl_loss"].item(), 1e-6, 1e-4, "kl_loss")
    gm = newr.grad.abs().max().item()
    close(nd.grad, newr.grad.numpy(), 1e-6 * gm, 1e-4, "dlp 512x1024")


def test_headline_dual_clip_lower_branch_512x1024_loss_micro_batches():
    """the timed bench step (old = recomputed + N(0, 0.05^2)) fires the
    dual-clip lower branch 0 times in 10.49M tokens, so here the bench's batch shape and loss
    micro-batching (512 x 1,024, GRPO advantages of groups of 8, 64 segments of the reference's
    ppo_micro_batch_size_per_gpu = 8 rows, token-mean each, k3 KL) with old = new + 0.5 N(0, 1): the
    ratio passes clip_ratio_c = 3 on negative advantages (core_algos.py:785-791) for a few percent of
    the tokens. Every segment's pg_loss, clipfrac, ppo_kl, clipfrac_lower and kl_loss and the
    accumulated gradient d(sum_s loss_s / 64) / d log_prob against the oracle's 64 separate
    micro-batch losses (dp_actor.py:419-470)."""
    from verl_amd import kernels as K
    from verl_amd.trainer.ppo import core_algos

    g = torch.Generator().manual_seed(606)
    B, R, S = 512, 1024, 8
    lens = torch.randint(128, R + 1, (B,), generator=g)
    mask = (torch.arange(R)[None, :] < lens[:, None]).long()
    rewards = torch.zeros(B, R)
    rewards[torch.arange(B), lens - 1] = torch.bernoulli(torch.full((B,), 0.5), generator=g)
    uid = np.array([f"p{i // 8}" for i in range(B)], dtype=object)
    adv, _ = ref.compute_grpo_outcome_advantage(rewards.clone(), mask, uid)
    new = -torch.rand(B, R, generator=g) * 3
    old = new + 0.5 * torch.randn(B, R, generator=g)
    refl = new + 0.1 * torch.randn(B, R, generator=g)
    nseg = B // S
    newr = new.clone().requires_grad_(True)
    want = []
    total = 0.0
    for i in range(nseg):
        sl = slice(i * S, (i + 1) * S)
        loss, met = ref.actor_loss(old[sl], newr[sl], adv[sl], mask[sl], clip_ratio=0.2, clip_ratio_c=3.0,
                                   ref_log_prob=refl[sl], kl_loss_type="low_var_kl", kl_loss_coef=0.001,
                                   grad_scale=1.0 / nseg)
        total = total + loss
        want.append([met["pg_loss"].item(), met["pg_clipfrac"].item(), met["ppo_kl"].item(),
                     met["pg_clipfrac_lower"].item(), met["kl_loss"].item()])
    total.backward()
    want = np.asarray(want)
    assert (want[:, 3] > 0).sum() >= nseg // 2, "the lower branch must fire in most segments"
    nd = new.to(DEV).requires_grad_(True)
    out = K.fused_policy_loss(old.to(DEV), nd, adv.to(DEV), mask.to(DEV), 0.2, 0.2, 3.0, "token-mean",
                              ref_log_prob=refl.to(DEV), kl_loss_type="low_var_kl", seg_rows=S)
    assert tuple(out.shape) == (nseg, 8)
    ((out[:, 0] + 0.001 * out[:, 4]).sum() / nseg).backward()
    got = out[:, [0, 1, 2, 3, 4]].detach().cpu().double().numpy()
    clipped_lower_tokens = (got[:, 3] * out[:, 6].detach().cpu().double().numpy()).sum()
    assert clipped_lower_tokens > 1000, clipped_lower_tokens
    np.testing.assert_allclose(got[:, 0], want[:, 0], atol=1e-5, rtol=1e-4, err_msg="pg_loss per segment")
    np.testing.assert_allclose(got[:, 1], want[:, 1], atol=1e-6, rtol=1e-6, err_msg="clipfrac")
    np.testing.assert_allclose(got[:, 3], want[:, 3], atol=1e-6, rtol=1e-6, err_msg="clipfrac_lower")
    np.testing.assert_allclose(got[:, 2], want[:, 2], atol=1e-6, rtol=1e-4, err_msg="ppo_kl")
    np.testing.assert_allclose(got[:, 4], want[:, 4], atol=1e-6, rtol=1e-4, err_msg="kl_loss")
    gm = newr.grad.abs().max().item()
    close(nd.grad, newr.grad.numpy(), 1e-6 * gm, 1e-4, "accumulated dlp with the lower branch")


def test_headline_logprob_micro_batch_8x1024x151936():
    """A full update micro-batch of logits (8 x 1024 rows x 151,936 bf16 = 2.5 GB): oracle on 64
    sampled rows; on all rows the size-independent invariants logp <= 0, 0 <= H <= log V, and
    fwd/bwd consistency: sum_j dlogits[i, j] = 0 for the log-prob gradient (softmax rows sum to 1)."""
    from verl_amd import kernels as K

    n, V = 8 * 1024, 151936
    torch.manual_seed(0)
    logits = (torch.randn(n, V, device=DEV) * 2).to(torch.bfloat16)
    labels = torch.randint(0, V, (n,), device=DEV)
    x = logits.clone().requires_grad_(True)
    lp, ent = K.logprob_entropy(x, labels)
    assert torch.all(lp <= 0) and torch.all(ent >= 0) and torch.all(ent <= np.log(V) + 1e-4)
    rows = torch.randperm(n)[:64]
    sub = logits[rows.to(DEV)].cpu()
    close(lp[rows.to(DEV)], ref.logprobs_fp32_math(sub, labels[rows.to(DEV)].cpu()).numpy(), 1e-4, 1e-4, "logp rows")
    close(ent[rows.to(DEV)], ref.entropy_from_logits(sub.float()).numpy(), 1e-4, 1e-4, "entropy rows")
    lp.sum().backward()
    rowsum = x.grad.float().sum(dim=-1)
    assert rowsum.abs().max().item() < 5e-2  # bf16-rounded gradients of onehot - softmax


def test_bench_logprob_launch_131072x151936():
    """The bench's own log-prob launch (micro-batch 128 x 1024 response rows x 151,936 bf16 = 40 GB,
    2.49e9 16-B vectors: past 2^31, so the flat backward's 64-bit indexing is exercised): oracle on
    sampled rows incl. the first and last, row-sum invariant on every row, and the flat backward
    bitwise equal to the per-row-chunk backward. Peak ~120 GB of HBM."""
    from verl_amd import _lib as L
    from verl_amd import kernels as K

    n, V = 128 * 1024, 151936
    gen = torch.Generator(device=DEV).manual_seed(5)
    x = torch.randn(n, V, device=DEV, dtype=torch.bfloat16, generator=gen).mul_(2)
    labels = torch.randint(0, V, (n,), device=DEV, generator=gen)
    labels[-1] = V - 1
    lp, ent, lse = (torch.empty(n, device=DEV) for _ in range(3))
    st = K._stream(x)
    L.call("va_logprob_entropy_fwd", K._p(x), L.VA_BF16, n, V, V, K._p(labels), 1.0, K._p(lp), K._p(ent), K._p(lse), st)
    rows = torch.cat([torch.tensor([0, 1, n // 2, n - 2, n - 1]), torch.randperm(n)[:11]]).to(DEV)
    sub = x[rows].cpu()
    close(lp[rows], ref.logprobs_fp32_math(sub, labels[rows].cpu()).numpy(), 1e-4, 1e-4, "logp rows")
    close(ent[rows], ref.entropy_from_logits(sub.float()).numpy(), 1e-4, 1e-4, "entropy rows")
    g = torch.randn(n, device=DEV, generator=gen)
    dx = torch.empty_like(x)
    try:
        L.call("va_set_tuning", L.VA_TUNE_BWD_FLAT, -1)
        L.call("va_logprob_entropy_bwd", K._p(g), None, K._p(x), L.VA_BF16, n, V, V, K._p(labels), K._p(lse),
               K._p(ent), 1.0, K._p(dx), V, st)
        # oracle gradient of sum_i g_i logp_i on the sampled rows: g (onehot - softmax), float64
        p = torch.softmax(sub.double(), dim=-1)
        want = -p * g[rows].cpu().double()[:, None]
        want[torch.arange(len(rows)), labels[rows].cpu()] += g[rows].cpu().double()
        close(dx[rows], want.numpy(), 2e-3 * want.abs().max().item(), 1e-2, "dlogits rows")
        rowsum = dx.sum(dim=-1, dtype=torch.float32)
        assert rowsum.abs().max().item() < 5e-2 * g.abs().max().item()
        dx2 = torch.empty_like(x)
        L.call("va_set_tuning", L.VA_TUNE_BWD_FLAT, 0)
        L.call("va_logprob_entropy_bwd", K._p(g), None, K._p(x), L.VA_BF16, n, V, V, K._p(labels), K._p(lse),
               K._p(ent), 1.0, K._p(dx2), V, st)
        assert torch.equal(dx, dx2)
    finally:
        L.call("va_set_tuning", L.VA_TUNE_BWD_FLAT, -1)
