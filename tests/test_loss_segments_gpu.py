"""Loss micro-batch segments of the fused policy loss (va_ppo_loss_fwd/bwd, seg_rows > 0).

One [B, R] launch over S = ceil(B / seg_rows) of the reference's loss micro-batches must give,
for every segment, what a separate launch over that segment's rows gives (dp_actor.py:388-470:
agg_loss per micro-batch, each / gradient_accumulation): the same 8 output slots and, for the
same upstream gradients, bitwise the same d_lp / d_entropy (the per-token weights use the
segment's own token and row counts). Also checked against the oracle per segment."""

import pytest
import torch

from oracle import reference_ops as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _inputs(B, R, seed, mask_dtype=torch.int64):
    g = torch.Generator(device=DEV).manual_seed(seed)
    lp = -torch.rand(B, R, device=DEV, generator=g) * 3
    old = lp + 0.3 * torch.randn(B, R, device=DEV, generator=g)
    ref_lp = lp + 0.2 * torch.randn(B, R, device=DEV, generator=g)
    adv = torch.randn(B, R, device=DEV, generator=g)
    ent = torch.rand(B, R, device=DEV, generator=g) * 5
    lens = torch.randint(1, R + 1, (B,), device=DEV, generator=g)
    lens[3] = 0  # an empty response inside a segment
    mask = (torch.arange(R, device=DEV)[None, :] < lens[:, None]).to(mask_dtype)
    return old, lp, adv, mask, ref_lp, ent


def _bits_equal(a, b):
    return torch.equal(a.view(torch.int32), b.view(torch.int32))


def _loss(old, lp, adv, mask, ref_lp, ent, agg, seg_rows, kl="low_var_kl"):
    from verl_amd import kernels as K

    return K.fused_policy_loss(old, lp, adv, mask, 0.2, 0.28, 3.0, agg, ref_log_prob=ref_lp if kl else None,
                               kl_loss_type=kl, entropy=ent, seg_rows=seg_rows)


@pytest.mark.parametrize("agg", ["token-mean", "seq-mean-token-sum", "seq-mean-token-mean", "seq-mean-token-sum-norm"])
@pytest.mark.parametrize("B,R,seg", [(130, 1024, 8), (64, 256, 16), (24, 37, 5), (16, 1024, 1)])
@pytest.mark.parametrize("kl", ["low_var_kl", None])
def test_segments_equal_separate_calls(agg, B, R, seg, kl):
    from verl_amd import _lib as L

    old, lp, adv, mask, ref_lp, ent = _inputs(B, R, seed=B + R + seg)
    lp_a = lp.clone().requires_grad_(True)
    ent_a = ent.clone().requires_grad_(True)
    out = _loss(old, lp_a, adv, mask, ref_lp, ent_a, agg, seg, kl)
    S = -(-B // seg)
    assert out.shape == (S, L.VA_LOSS_NOUT)
    # per-segment upstream gradients, as the actor's sum over micro-batches of policy_loss / ga
    w = torch.rand(S, 3, device=DEV)
    (out[:, L.VA_LOSS_PG] * w[:, 0] + out[:, L.VA_LOSS_KL] * w[:, 1] - out[:, L.VA_LOSS_ENTROPY] * w[:, 2]).sum().backward()
    for s in range(S):
        sl = slice(s * seg, min(B, (s + 1) * seg))
        lp_b = lp[sl].clone().requires_grad_(True)
        ent_b = ent[sl].clone().requires_grad_(True)
        o = _loss(old[sl].contiguous(), lp_b, adv[sl].contiguous(), mask[sl].contiguous(), ref_lp[sl].contiguous(),
                  ent_b, agg, 0, kl)
        assert o.shape == (L.VA_LOSS_NOUT,)
        # (a 0-token row makes seq-mean-token-mean NaN, as the reference's 0 / 0: NaN on both sides)
        assert torch.allclose(out[s], o, rtol=1e-6, atol=1e-7, equal_nan=True), (s, out[s], o)
        (o[L.VA_LOSS_PG] * w[s, 0] + o[L.VA_LOSS_KL] * w[s, 1] - o[L.VA_LOSS_ENTROPY] * w[s, 2]).backward()
        # same per-token weights (segment token / row counts): bitwise equal gradients
        assert _bits_equal(lp_a.grad[sl], lp_b.grad), s
        assert _bits_equal(ent_a.grad[sl], ent_b.grad), s


@pytest.mark.parametrize("mask_dtype", [torch.int64, torch.bool, torch.float32])
def test_segments_match_oracle(mask_dtype):
    """Each segment's slots against the oracle's compute_policy_loss / agg_loss(kl_penalty) /
    agg_loss(entropy) over that segment's rows (fp32 restatement of core_algos.py)."""
    from verl_amd import _lib as L

    B, R, seg = 40, 512, 8
    old, lp, adv, mask, ref_lp, ent = _inputs(B, R, seed=11, mask_dtype=mask_dtype)
    out = _loss(old, lp, adv, mask, ref_lp, ent, "token-mean", seg)
    for s in range(B // seg):
        sl = slice(s * seg, (s + 1) * seg)
        m = mask[sl].float().cpu()
        pg, cf, kl, cfl = ref.compute_policy_loss(old[sl].cpu(), lp[sl].cpu(), adv[sl].cpu(), m, cliprange=0.2,
                                                  cliprange_low=0.2, cliprange_high=0.28, clip_ratio_c=3.0,
                                                  loss_agg_mode="token-mean")
        kl_loss = ref.agg_loss(ref.kl_penalty(lp[sl].cpu(), ref_lp[sl].cpu(), "low_var_kl"), m, "token-mean")
        ent_loss = ref.agg_loss(ent[sl].cpu(), m, "token-mean")
        got = out[s].cpu()
        for slot, want in [(L.VA_LOSS_PG, pg), (L.VA_LOSS_CLIPFRAC, cf), (L.VA_LOSS_PPO_KL, kl),
                           (L.VA_LOSS_CLIPFRAC_LOWER, cfl), (L.VA_LOSS_KL, kl_loss), (L.VA_LOSS_ENTROPY, ent_loss)]:
            assert torch.allclose(got[slot], want.float(), rtol=1e-4, atol=1e-5), (s, slot, got[slot], want)
        assert got[L.VA_LOSS_NTOKENS].item() == m.sum().item()
        assert got[L.VA_LOSS_NROWS].item() == seg


def test_seg_rows_at_least_b_is_one_aggregate():
    from verl_amd import _lib as L

    old, lp, adv, mask, ref_lp, ent = _inputs(12, 64, seed=3)
    a = _loss(old, lp, adv, mask, ref_lp, ent, "token-mean", 0)
    b = _loss(old, lp, adv, mask, ref_lp, ent, "token-mean", 12)
    c = _loss(old, lp, adv, mask, ref_lp, ent, "token-mean", 100)
    assert a.shape == b.shape == c.shape == (L.VA_LOSS_NOUT,)
    assert torch.equal(a, b) and torch.equal(a, c)


@pytest.mark.parametrize("agg", ["token-mean", "seq-mean-token-mean", "seq-mean-token-sum-norm"])
@pytest.mark.parametrize("B,R,seg", [(130, 1024, 8), (24, 37, 5)])
def test_value_loss_segments_equal_separate_calls(agg, B, R, seg):
    """The critic's fused value loss with loss micro-batch segments (dp_critic.py:218-242)."""
    from verl_amd import _lib as L
    from verl_amd import kernels as K

    old, lp, adv, mask, ref_lp, _ = _inputs(B, R, seed=7 + B)
    vals, rets = lp, ref_lp + adv
    vp_a = (vals + 0.4 * adv).requires_grad_(True)
    out = K.fused_value_loss(vp_a, vals, rets, mask, 0.5, agg, seg_rows=seg)
    S = -(-B // seg)
    assert out.shape == (S, L.VA_VLOSS_NOUT)
    w = torch.rand(S, 2, device=DEV)
    (out[:, L.VA_VLOSS_LOSS] * w[:, 0] + out[:, L.VA_VLOSS_VPRED_MEAN] * w[:, 1]).sum().backward()
    for s in range(S):
        sl = slice(s * seg, min(B, (s + 1) * seg))
        vp_b = vp_a.detach()[sl].clone().requires_grad_(True)
        o = K.fused_value_loss(vp_b, vals[sl].contiguous(), rets[sl].contiguous(), mask[sl].contiguous(), 0.5, agg)
        assert torch.allclose(out[s], o, rtol=1e-6, atol=1e-7, equal_nan=True), (s, out[s], o)
        (o[L.VA_VLOSS_LOSS] * w[s, 0] + o[L.VA_VLOSS_VPRED_MEAN] * w[s, 1]).backward()
        assert _bits_equal(vp_a.grad[sl], vp_b.grad), s


@pytest.mark.parametrize("sizes", [[3, 1, 7, 5], [16], [1] * 9, [2, 30, 2]])
def test_variable_segments_equal_separate_calls(sizes):
    """seg_off: segments of any sizes (the reference's token-budget micro-batches), policy and value
    loss, against separate launches over each segment's rows."""
    from verl_amd import _lib as L
    from verl_amd import kernels as K

    B, R = sum(sizes), 1024
    old, lp, adv, mask, ref_lp, ent = _inputs(max(B, 4), R, seed=len(sizes))
    old, lp, adv, mask, ref_lp, ent = (t[:B].contiguous() for t in (old, lp, adv, mask, ref_lp, ent))
    off = [0]
    for s in sizes:
        off.append(off[-1] + s)
    lp_a = lp.clone().requires_grad_(True)
    out = K.fused_policy_loss(old, lp_a, adv, mask, 0.2, 0.28, 3.0, "seq-mean-token-sum", ref_log_prob=ref_lp,
                              kl_loss_type="low_var_kl", seg_off=off)
    vp_a = (lp + 0.3).requires_grad_(True)
    vout = K.fused_value_loss(vp_a, lp, ref_lp, mask, 0.5, "token-mean", seg_off=off)
    S = len(sizes)
    assert out.shape == (S, L.VA_LOSS_NOUT) and vout.shape == (S, L.VA_VLOSS_NOUT)
    w = torch.rand(S, 3, device=DEV)
    (out[:, L.VA_LOSS_PG] * w[:, 0] + out[:, L.VA_LOSS_KL] * w[:, 1] + vout[:, L.VA_VLOSS_LOSS] * w[:, 2]).sum().backward()
    for s in range(S):
        sl = slice(off[s], off[s + 1])
        lp_b = lp[sl].clone().requires_grad_(True)
        o = K.fused_policy_loss(old[sl].contiguous(), lp_b, adv[sl].contiguous(), mask[sl].contiguous(), 0.2, 0.28, 3.0,
                                "seq-mean-token-sum", ref_log_prob=ref_lp[sl].contiguous(), kl_loss_type="low_var_kl")
        vp_b = (lp[sl] + 0.3).requires_grad_(True)
        vo = K.fused_value_loss(vp_b, lp[sl].contiguous(), ref_lp[sl].contiguous(), mask[sl].contiguous(), 0.5,
                                "token-mean")
        assert torch.allclose(out[s], o, rtol=1e-6, atol=1e-7, equal_nan=True), (s, out[s], o)
        assert torch.allclose(vout[s], vo, rtol=1e-6, atol=1e-7, equal_nan=True), (s, vout[s], vo)
        (o[L.VA_LOSS_PG] * w[s, 0] + o[L.VA_LOSS_KL] * w[s, 1] + vo[L.VA_VLOSS_LOSS] * w[s, 2]).backward()
        assert _bits_equal(lp_a.grad[sl], lp_b.grad), s
        assert _bits_equal(vp_a.grad[sl], vp_b.grad), s
