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
