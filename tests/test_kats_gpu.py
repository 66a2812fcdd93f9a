"""The HIP kernels against answers worked out by hand from the reference source (tests/kat_cases.py),
so the kernels are pinned directly, not only through the CPU oracle."""

import numpy as np
import pytest
import torch

from tests import kat_cases as C

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _t(x, dtype=torch.float32):
    return torch.tensor(x, dtype=dtype, device=DEV)


@pytest.mark.parametrize("shape", [(1, 4), (4, 1), (2, 2)])
@pytest.mark.parametrize("mask_dtype", [torch.int64, torch.float32, torch.bool])
def test_dual_clip_policy_loss_kernel_hand_kat(shape, mask_dtype):
    from verl_amd import _lib as L
    from verl_amd import kernels as K

    c = C.POLICY_CASE
    lp = _t(c["d_lp"]).view(shape).clone().requires_grad_(True)
    out = K.fused_policy_loss(_t([0.0] * 4).view(shape), lp, _t(c["adv"]).view(shape),
                              torch.ones(shape, dtype=mask_dtype, device=DEV), 0.2, 0.2, 3.0, "token-mean")
    got = out.detach().cpu()
    assert abs(got[L.VA_LOSS_PG].item() - c["pg_loss"]) < 1e-6
    assert abs(got[L.VA_LOSS_CLIPFRAC].item() - c["clipfrac"]) < 1e-7
    assert abs(got[L.VA_LOSS_CLIPFRAC_LOWER].item() - c["clipfrac_lower"]) < 1e-7
    assert abs(got[L.VA_LOSS_PPO_KL].item() - c["ppo_kl"]) < 1e-6
    out[L.VA_LOSS_PG].backward()
    assert torch.allclose(lp.grad.view(-1).cpu(), torch.tensor(c["dlp"]), atol=1e-7)
    c = C.CLAMP_CASE
    out = K.fused_policy_loss(_t([[0.0]]), _t([c["d_lp"]]), _t([c["adv"]]), torch.ones(1, 1, device=DEV), 0.2, 0.2,
                              3.0, "token-mean").cpu()
    got = (out[L.VA_LOSS_PG].item(), out[L.VA_LOSS_CLIPFRAC].item(), out[L.VA_LOSS_CLIPFRAC_LOWER].item(),
           out[L.VA_LOSS_PPO_KL].item())
    assert np.allclose(got, (c["pg_loss"], c["clipfrac"], c["clipfrac_lower"], c["ppo_kl"]), rtol=1e-6, atol=0)


def test_agg_kl_whiten_grpo_kernel_hand_kats():
    from verl_amd.trainer.ppo import core_algos
    from verl_amd.utils import torch_functional as vF

    for mode, want in C.AGG_WANT.items():
        got = core_algos.agg_loss(_t(C.AGG_LOSS), _t(C.AGG_MASK, torch.int64), mode).item()
        assert abs(got - want) < 1e-6, mode
    for kt, want in C.KL_WANT.items():
        got = core_algos.kl_penalty(_t(C.KL_LP), _t(C.KL_REF), kt).cpu()
        assert torch.allclose(got, torch.tensor(want), atol=1e-6, rtol=1e-6), kt
    got = vF.masked_whiten(_t(C.WHITEN_X).view(1, -1), _t(C.WHITEN_MASK, torch.int64).view(1, -1)).view(-1).cpu()
    assert torch.allclose(got, torch.tensor(C.WHITEN_WANT), atol=1e-5)
    rew = torch.zeros(5, 4, device=DEV)
    rew[:, 1] = _t(C.GRPO_SCORES)
    mask = torch.ones(5, 4, dtype=torch.int64, device=DEV)
    uid = np.array(C.GRPO_UID, dtype=object)
    adv, _ = core_algos.compute_grpo_outcome_advantage(rew, mask, uid)
    assert torch.allclose(adv[:, 0].cpu(), torch.tensor(C.GRPO_WANT), atol=1e-5)
    adv, _ = core_algos.compute_grpo_outcome_advantage(rew, mask, uid, norm_adv_by_std_in_grpo=False)
    assert torch.allclose(adv[:, 0].cpu(), torch.tensor(C.GRPO_NOSTD_WANT), atol=1e-6)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("temperature", [1.0, 2.0])
def test_logprob_entropy_kernel_closed_form(dtype, temperature):
    """va_logprob_entropy_fwd / _bwd against the closed forms of tests/kat_cases.py (two-level rows,
    exact in bf16): logp and entropy to fp32 rounding; dlogits to 1e-5 relative (fp32 logits) or to
    one bf16 rounding (bf16 logits: the gradient is written in the logits' dtype)."""
    from verl_amd import kernels as K

    rows, labels = C.ls_logits()
    x = torch.tensor(rows, dtype=dtype, device=DEV).requires_grad_(True)
    lab = torch.tensor(labels, device=DEV)
    lp, ent = K.logprob_entropy(x, lab, temperature, inplace_backward=False)
    want_lp, want_ent, want_g = C.ls_expected(temperature, g_logp=1.0, g_ent=0.5)
    assert torch.allclose(lp.cpu().double(), torch.tensor(want_lp, dtype=torch.float64), atol=2e-6, rtol=0)
    assert torch.allclose(ent.cpu().double(), torch.tensor(want_ent, dtype=torch.float64), atol=2e-6, rtol=0)
    (lp.sum() + 0.5 * ent.sum()).backward()
    g = torch.tensor(want_g, dtype=torch.float64)
    tol = 1e-5 if dtype == torch.float32 else 2.0 ** -8  # fp32: v_exp_f32 (1 ulp) inside p
    assert torch.allclose(x.grad.cpu().double(), g, atol=1e-9, rtol=tol)


@pytest.mark.parametrize("fp32_logits", [False, True])
@pytest.mark.parametrize("temperature", [1.0, 2.0])
def test_fused_lm_head_kernel_closed_form(fp32_logits, temperature):
    """f1 (va_linear_logprob_fwd and the fused vocab-range backward) on a hidden / weight pair whose
    product is exactly the two-level rows of tests/kat_cases.py: hidden row r = c_r e_r, weight[j, r] =
    [j < k_r]. logp / entropy to fp32 rounding; d hidden = dlogits W and d weight = dlogits^T hidden from
    the closed-form dlogits rounded to bf16 (the dtype the fused backward writes them in)."""
    from verl_amd import kernels as K

    n, H = len(C.LS_ROWS), 64
    hid = torch.zeros(n, H, dtype=torch.float64)
    w = torch.zeros(C.LS_V, H, dtype=torch.float64)
    for r, (k, c, _) in enumerate(C.LS_ROWS):
        hid[r, r] = c
        w[:k, r] = 1.0
    labels = torch.tensor([lab for _, _, lab in C.LS_ROWS], device=DEV)
    hb = hid.to(torch.bfloat16).to(DEV).requires_grad_(True)
    wb = w.to(torch.bfloat16).to(DEV).requires_grad_(True)
    lp, ent = K.linear_logprob_entropy(hb, wb, labels, temperature, fp32_logits=fp32_logits)
    want_lp, want_ent, want_g = C.ls_expected(temperature, g_logp=1.0, g_ent=0.5)
    assert torch.allclose(lp.detach().cpu().double(), torch.tensor(want_lp, dtype=torch.float64), atol=2e-6, rtol=0)
    assert torch.allclose(ent.detach().cpu().double(), torch.tensor(want_ent, dtype=torch.float64), atol=2e-6, rtol=0)
    (lp.sum() + 0.5 * ent.sum()).backward()
    g = torch.tensor(want_g, dtype=torch.float64).to(torch.bfloat16).double()  # the fused backward's dlogits are bf16
    want_dh, want_dw = g @ w, g.t() @ hid
    # the two GEMMs run in bf16 with fp32 accumulation and a bf16 result
    for got, want, what in ((hb.grad, want_dh, "d hidden"), (wb.grad, want_dw, "d weight")):
        got = got.cpu().double()
        err = ((got - want).abs() - 2.0 ** -7 * want.abs()).max().item()
        assert err <= 1e-6, f"{what}: {err:.3e} beyond one bf16 rounding"


@pytest.mark.parametrize("R", [3, 8])
def test_estimator_kernels_hand_kats(R):
    """RLOO / OPO / pass@k / REINFORCE++ / ReMax / GAE kernels against tests/kat_cases.py (R = 3: the
    unaligned-row kernels; R = 8: the 16-byte quad kernels, the extra columns masked out)."""
    from verl_amd.trainer.ppo import core_algos
    from verl_amd.utils.config import AttrDict

    def col(scores, lengths=None):
        rew = torch.zeros(len(scores), R, device=DEV)
        rew[:, 0] = _t(scores)
        mask = torch.ones(len(scores), R, dtype=torch.int64, device=DEV)
        if lengths is not None:
            for i, n in enumerate(lengths):
                mask[i, n:] = 0
        return rew, mask

    def pad(rows, fill=0.0):
        return _t([list(r) + [fill] * (R - len(r)) for r in rows])

    uid = lambda u: np.array(u, dtype=object)  # noqa: E731
    rew, mask = col(C.RLOO_SCORES)
    adv, _ = core_algos.compute_rloo_outcome_advantage(rew, mask, uid(C.RLOO_UID))
    assert torch.allclose(adv[:, 0].cpu(), torch.tensor(C.RLOO_WANT), atol=1e-6)
    rew, mask = col(C.OPO_SCORES, lengths=C.OPO_LEN)
    adv, _ = core_algos.compute_opo_outcome_advantage(rew, mask, uid(C.OPO_UID))
    assert torch.allclose(adv[:, 0].cpu(), torch.tensor(C.OPO_WANT), atol=1e-6)
    assert torch.count_nonzero(adv[mask == 0]).item() == 0
    rew, mask = col(C.PASSK_SCORES)
    for norm, want in ((True, C.PASSK_WANT), (False, C.PASSK_NOSTD_WANT)):
        adv, _ = core_algos.compute_grpo_passk_outcome_advantage(
            rew, mask, uid(C.PASSK_UID), config=AttrDict(norm_adv_by_std_in_grpo=norm))
        assert torch.allclose(adv[:, 0].cpu(), torch.tensor(want), atol=1e-6), norm
    m = pad(C.RFPP_MASK).to(torch.int64)
    adv, ret = core_algos.compute_reinforce_plus_plus_outcome_advantage(pad(C.RFPP_REWARDS), m,
                                                                        config=AttrDict(gamma=0.5))
    assert torch.allclose(ret[:, :3].cpu(), torch.tensor(C.RFPP_RETURNS), atol=1e-6)
    assert torch.allclose(adv[:, :3].cpu(), torch.tensor(C.RFPP_ADV), atol=1e-5)
    assert torch.count_nonzero(adv[m == 0]).item() == 0
    if R >= 4:
        m = pad(C.REMAX_MASK).to(torch.int64)
        adv, ret = core_algos.compute_remax_outcome_advantage(pad(C.REMAX_REWARDS), _t(C.REMAX_BASE), m,
                                                              config=AttrDict(gamma=1.0))
        assert torch.allclose(ret[:, :4].cpu(), torch.tensor(C.REMAX_RETURNS), atol=1e-7)
        assert torch.allclose(adv[:, :4].cpu(), torch.tensor(C.REMAX_ADV), atol=1e-7)
    adv, ret = core_algos.compute_gae_advantage_return(pad(C.GAE_REWARDS), pad(C.GAE_VALUES),
                                                       pad(C.GAE_MASK).to(torch.int64), 0.5, 0.5)
    assert torch.allclose(ret[:, :3].cpu(), torch.tensor(C.GAE_RETURNS), atol=1e-6)
    assert torch.allclose(adv[:, :3].cpu(), torch.tensor(C.GAE_ADV), atol=1e-5)


def test_loss_variant_kernels_hand_kats():
    """gpg / kl_cov / clip_cov through the registered loss functions (selection on the host, loss and
    gradient in the fused kernel) against tests/kat_cases.py."""
    from verl_amd.trainer.ppo import core_algos
    from verl_amd.utils.config import actor_config

    cfg = actor_config()
    cfg.policy_loss.kl_cov_ratio = 0.25
    cfg.policy_loss.ppo_kl_coef = 1.0
    cfg.policy_loss.clip_cov_ratio = 0.25
    cfg.policy_loss.clip_cov_lb = 1.0
    cfg.policy_loss.clip_cov_ub = 5.0
    m = torch.ones(1, 4, dtype=torch.int64, device=DEV)
    adv = _t([C.GPG_ADV])

    def run(name, old, lp_vals, a):
        lp = _t([lp_vals]).requires_grad_(True)
        out = core_algos.get_policy_loss_fn(name)(old, lp, a, m, "token-mean", cfg)
        out[0].backward()
        return [o.item() for o in out], lp.grad[0].cpu()

    (loss, cf, kl, cfl), g = run("gpg", torch.zeros(1, 4, device=DEV), C.GPG_LP, adv)
    assert abs(loss - C.GPG_LOSS) < 1e-6 and (cf, kl, cfl) == (0.0, 0.0, 0.0)
    assert torch.allclose(g, torch.tensor(C.GPG_DLP), atol=1e-7)
    (loss, cf, kl, cfl), g = run("kl_cov", torch.zeros(1, 4, device=DEV), C.GPG_LP, adv)
    assert abs(loss - C.KLCOV_LOSS) < 1e-6 and abs(kl - C.KLCOV_PPO_KL) < 1e-6
    assert torch.allclose(g, torch.tensor(C.KLCOV_DLP), atol=1e-6)
    (loss, cf, kl, cfl), g = run("clip_cov", _t([C.CLIPCOV_LP]), C.CLIPCOV_LP, _t([C.CLIPCOV_ADV]))
    assert abs(loss - C.CLIPCOV_LOSS) < 1e-6 and abs(cf - C.CLIPCOV_CLIPFRAC) < 1e-6 and kl == 0.0
    assert torch.allclose(g, torch.tensor(C.CLIPCOV_DLP), atol=1e-7)


def test_value_loss_kernel_hand_kat():
    """core_algos.py:992-1031 by hand (the oracle's test_value_loss_kats): values 0, cliprange 0.5,
    vpreds 2 -> clipped 0.5; returns 0: (2 - 0)^2 = 4 vs (0.5 - 0)^2 = 0.25 -> 4 (unclipped wins);
    returns 3: 1 vs 6.25 -> 6.25 (clipped wins). loss = 0.5 mean = 0.5 (4 + 6.25) / 2, clipfrac 1/2;
    d loss / d vpreds = 0.5 * 2 (2 - 0) / 2 for token 0 and 0 for token 1 (the clipped branch is flat)."""
    from verl_amd.trainer.ppo import core_algos

    vp = _t([[2.0, 2.0]]).requires_grad_(True)
    loss, frac = core_algos.compute_value_loss(vp, _t([[0.0, 3.0]]), _t([[0.0, 0.0]]),
                                               torch.ones(1, 2, dtype=torch.int64, device=DEV), 0.5)
    loss.backward()
    assert abs(loss.item() - 0.5 * (4.0 + 6.25) / (2 + 1e-8)) < 1e-6
    assert abs(frac.item() - 1 / (2 + 1e-8)) < 1e-7
    assert torch.allclose(vp.grad.cpu(), torch.tensor([[2.0 / (2 + 1e-8), 0.0]]), atol=1e-6)


def test_group_estimators_on_an_empty_batch():
    """B = 0: the reference's group loops do not run (core_algos.py:282-308, 311-370, 428-667), so
    GRPO / Dr.GRPO / pass@k / RLOO / OPO / GPG / ReMax return empty [0, R] advantages; RF++-baseline,
    RF++ and GAE reach masked_whiten with an all-zero mask and raise its ValueError."""
    from verl_amd.trainer.ppo import core_algos
    from verl_amd.utils.config import AttrDict

    r = torch.zeros(0, 8, device=DEV)
    m = torch.zeros(0, 8, dtype=torch.int64, device=DEV)
    idx = np.array([], dtype=object)
    outs = [core_algos.compute_grpo_outcome_advantage(r, m, idx),
            core_algos.compute_grpo_outcome_advantage(r, m, idx, norm_adv_by_std_in_grpo=False),
            core_algos.compute_grpo_passk_outcome_advantage(r, m, idx, config=AttrDict(norm_adv_by_std_in_grpo=True)),
            core_algos.compute_rloo_outcome_advantage(r, m, idx),
            core_algos.compute_opo_outcome_advantage(r, m, idx),
            core_algos.compute_gpg_outcome_advantage(r, m, idx)]
    for adv, ret in outs:
        assert adv.shape == (0, 8) and ret.shape == (0, 8) and adv.dtype == torch.float32
    adv, ret = core_algos.compute_remax_outcome_advantage(r, torch.zeros(0, device=DEV), m, config=AttrDict(gamma=1.0))
    assert adv.shape == (0, 8) and ret.shape == (0, 8)
    for fn in (lambda: core_algos.compute_reinforce_plus_plus_baseline_outcome_advantage(r, m, idx),
               lambda: core_algos.compute_reinforce_plus_plus_outcome_advantage(r, m, config=AttrDict(gamma=1.0)),
               lambda: core_algos.compute_gae_advantage_return(r, r, m, 1.0, 1.0)):
        with pytest.raises(ValueError, match="At least one element in the mask has to be 1"):
            fn()


def test_agg_loss_fully_masked_row():
    """agg_loss with a row whose mask is all 0 (core_algos.py:686-719): token-mean and the sum modes
    ignore it, seq-mean-token-mean divides 0 by 0 for it and returns NaN, as torch does."""
    from verl_amd.trainer.ppo import core_algos

    x = _t([[1.0, 2.0, 3.0], [4.0, 5.0, 6.0]])
    m = _t([[1, 1, 0], [0, 0, 0]], torch.int64)
    assert abs(core_algos.agg_loss(x, m, "token-mean").item() - 3.0 / (2 + 1e-8)) < 1e-6
    assert core_algos.agg_loss(x, m, "seq-mean-token-sum").item() == 1.5
    assert core_algos.agg_loss(x, m, "seq-mean-token-sum-norm").item() == 1.0
    assert torch.isnan(core_algos.agg_loss(x, m, "seq-mean-token-mean")).item()
