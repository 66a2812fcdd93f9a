"""torch.library registration of the hot-path kernels:
torch.library.opcheck on every torch.ops.verl_amd op (schema, fake/meta kernel, autograd
registration, AOT dispatch), and torch.compile(fullgraph=True) over the reference's log-prob +
actor-loss composition (the reference compiles entropy_from_logits, dp_actor.py:74-75) with no
graph breaks and results bitwise equal to eager."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
ops = torch.ops.verl_amd


@pytest.fixture(scope="module", autouse=True)
def _registered():
    from verl_amd import custom_ops, kernels  # noqa: F401


def _inputs(B=4, R=96, V=1000, seed=0):
    g = torch.Generator().manual_seed(seed)
    logits = (torch.randn(B * R, V, generator=g) * 2).to(torch.bfloat16)
    labels = torch.randint(0, V, (B * R,), generator=g)
    old = -torch.rand(B, R, generator=g) * 3
    adv = torch.randn(B, R, generator=g)
    lens = torch.randint(1, R + 1, (B,), generator=g)
    mask = (torch.arange(R)[None, :] < lens[:, None]).long()
    ref = old + 0.1 * torch.randn(B, R, generator=g)
    return [t.to(DEV) for t in (logits, labels, old, adv, mask, ref)]


def _check(op, args, **kw):
    torch.library.opcheck(op, args, **kw)


def test_opcheck_logprob_entropy():
    logits, labels, *_ = _inputs()
    x = logits.clone().requires_grad_(True)
    _check(ops.logprob_entropy_fwd, (x, labels, 1.0, False))
    _check(ops.logprob_entropy_fwd, (logits.float().requires_grad_(True), labels, 0.7, False))
    logp, ent, lse = ops.logprob_entropy_fwd(logits, labels, 1.0, 0)
    g = torch.randn_like(logp)
    _check(ops.logprob_entropy_bwd, (g, g, logits, labels, lse, ent, 1.0))
    _check(ops.logprob_entropy_bwd, (g, None, logits, labels, lse, ent, 1.0))
    _check(ops.logprob_entropy_bwd_, (g, g, logits.clone(), labels, lse, ent, 1.0))


@pytest.mark.parametrize("mode,kl,seg", [(0, 3, 0), (0, -1, 0), (1, 0, 0), (2, 3, 0), (3, 1, 0), (0, 3, 3)])
def test_opcheck_ppo_loss(mode, kl, seg):
    B = 8 if seg else 4  # seg 3: loss micro-batches of rows [0:3], [3:6], [6:8] -> out [3, 8]
    _, _, old, adv, mask, ref = _inputs(B=B)
    lp = (old + 0.05 * torch.randn_like(old)).requires_grad_(True)
    ent = torch.rand_like(old).requires_grad_(True)
    sel = (torch.rand_like(old) < 0.1).to(torch.uint8) if mode in (2, 3) else None
    args = (old, lp, adv, mask, ref if kl >= 0 else None, ent, sel, 0.8, 1.2, 3.0, 0, kl, mode, 0.1, seg)
    _check(ops.ppo_loss_fwd, args)
    out, ws = ops.ppo_loss_fwd(*args)
    assert out.shape == ((3, 8) if seg else (8,))
    g = torch.ones_like(out)
    _check(ops.ppo_loss_bwd, (g, old, lp.detach(), adv, mask, args[4], sel, ws, 0.8, 1.2, 3.0, 0, kl, mode, 0.1, True,
                              seg))
    if seg:  # the same 3 segments as row offsets
        off = torch.tensor([0, 2, 3, 8], dtype=torch.int32, device=DEV)
        args = args[:-1] + (0, off)
        _check(ops.ppo_loss_fwd, args)
        out, ws = ops.ppo_loss_fwd(*args)
        _check(ops.ppo_loss_bwd, (torch.ones_like(out), old, lp.detach(), adv, mask, args[4], sel, ws, 0.8, 1.2, 3.0, 0,
                                  kl, mode, 0.1, True, 0, off))


def test_opcheck_kl_agg_value():
    _, _, old, adv, mask, ref = _inputs()
    lp = old.clone().requires_grad_(True)
    for kt in (0, 1, 2, 3):
        _check(ops.kl_penalty_fwd, (lp, ref, kt))
        _check(ops.kl_penalty_bwd, (torch.randn_like(old), old, ref, kt))
    x = adv.clone().requires_grad_(True)
    for mode in (0, 1, 2, 3, 4, 5):
        _check(ops.masked_agg_fwd, (x, mask, mode))
        out, ws = ops.masked_agg_fwd(adv, mask, mode)
        _check(ops.masked_agg_bwd, (torch.ones_like(out), mask, mode, ws))
    vp = (old + 0.3 * torch.randn_like(old)).requires_grad_(True)
    _check(ops.value_loss_fwd, (vp, old, ref, mask, 0.5, 0))
    out, ws = ops.value_loss_fwd(vp.detach(), old, ref, mask, 0.5, 0)
    _check(ops.value_loss_bwd, (torch.ones_like(out), vp.detach(), old, ref, mask, ws, 0.5, 0))
    # two loss micro-batches of 2 rows: out [2, 4]
    _check(ops.value_loss_fwd, (vp, old, ref, mask, 0.5, 0, 2))
    out, ws = ops.value_loss_fwd(vp.detach(), old, ref, mask, 0.5, 0, 2)
    assert out.shape == (2, 4)
    _check(ops.value_loss_bwd, (torch.ones_like(out), vp.detach(), old, ref, mask, ws, 0.5, 0, 2))


def test_opcheck_advantage_ops():
    from verl_amd import _lib as L
    from verl_amd import kernels as K

    _, _, old, adv, mask, ref = _inputs(B=16)
    rewards = torch.zeros_like(old)
    rewards[:, -1] = torch.randn(16, device=DEV)
    index = np.array([f"u{i % 4}" for i in range(16)], dtype=object)
    order, offsets, G, gmax = K.group_csr(index, DEV)
    for est in (L.VA_ADV_GRPO, L.VA_ADV_RLOO, L.VA_ADV_OPO, L.VA_ADV_PASSK):
        _check(ops.outcome_advantage, (rewards, mask, order, offsets, G, gmax, 1e-6, est))
    _check(ops.row_scores, (rewards, mask, True))
    _check(ops.row_scores, (rewards, None, False))
    scores, lens = ops.row_scores(rewards, mask, True)
    _check(ops.group_coef, (scores, lens, order, offsets, G, gmax, 1e-6, L.VA_ADV_OPO))
    _check(ops.broadcast_rows, (scores, mask))
    values = torch.randn_like(old)
    _check(ops.gae_scan, (rewards, values, mask, 0.99, 0.95))
    _check(ops.gae_advantage_return, (rewards, values, mask, 0.99, 0.95))
    part = ops.masked_row_partials(adv, mask)
    _check(ops.masked_row_partials, (adv, mask))
    _check(ops.whiten_finalize, (part, 16))
    _, stats = ops.whiten_finalize(part, 16)
    _check(ops.whiten_apply, (adv, stats, mask, True))
    _check(ops.whiten_apply, (adv, stats, None, False))
    _check(ops.apply_kl_penalty, (rewards, old, ref, mask, 3, 0.01))
    _check(ops.discounted_returns, (rewards, mask, 0.99, L.VA_RET_RFPP, None))
    _check(ops.discounted_returns, (rewards, mask, 1.0, L.VA_RET_REMAX, torch.randn(16, device=DEV)))


def _actor_loss_fn(logits, labels, old, adv, mask, ref):
    from verl_amd.trainer.ppo import core_algos
    from verl_amd.utils import torch_functional as verl_F

    B, R = old.shape
    lp, ent = verl_F.logprobs_and_entropy_from_logits(logits, labels, 1.0, inplace_backward=False)
    return core_algos.compute_actor_loss(old, lp.view(B, R), adv, mask, 0.2, 0.28, 3.0, "token-mean",
                                         entropy=ent.view(B, R), ref_log_prob=ref, kl_loss_type="low_var_kl")


@pytest.mark.parametrize("backend", ["aot_eager", "inductor"])
def test_torch_compile_fullgraph_matches_eager_bitwise(backend):
    import torch._dynamo

    logits, labels, old, adv, mask, ref = _inputs(B=8, R=128, V=151936 // 8)
    old = old + 0.05 * torch.randn_like(old)  # ratios on both sides of the clip band
    torch._dynamo.reset()
    expl = torch._dynamo.explain(_actor_loss_fn)(logits, labels, old, adv, mask, ref)
    assert expl.graph_break_count == 0, expl.break_reasons
    x_e = logits.clone().requires_grad_(True)
    out_e = _actor_loss_fn(x_e, labels, old, adv, mask, ref)
    out_e.sum().backward()
    compiled = torch.compile(_actor_loss_fn, fullgraph=True, backend=backend)
    x_c = logits.clone().requires_grad_(True)
    out_c = compiled(x_c, labels, old, adv, mask, ref)
    out_c.sum().backward()
    assert torch.equal(out_c, out_e)
    assert torch.equal(x_c.grad, x_e.grad)
