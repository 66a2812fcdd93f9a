"""Fused bf16 model ops (RMSNorm / SwiGLU / RoPE) vs the HF Qwen2 modules they replace, and the
patched packed actor path vs the unpatched one."""

import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ulp_close(a, b, n_ulp=2, what=""):
    a, b = a.float(), b.float()
    tol = n_ulp * (2.0 ** -8) * b.abs() + 1e-6
    bad = (a - b).abs() > tol
    frac = bad.float().mean().item()
    assert frac < 1e-3, f"{what}: {frac:.2e} of elements beyond {n_ulp} bf16 ulp, max {(a - b).abs().max().item():.3e}"


def _grad_close(a, b, what, rtol=3e-2):
    a, b = a.float(), b.float()
    err = (a - b).norm() / (b.norm() + 1e-12)
    assert err < rtol, f"{what}: relative L2 error {err:.3e}"


def test_rmsnorm_matches_hf():
    from transformers.models.qwen2.modeling_qwen2 import Qwen2RMSNorm

    from verl_amd import kernels as K

    torch.manual_seed(0)
    T, H = 1000, 896
    m = Qwen2RMSNorm(H, eps=1e-6).to(DEV).to(torch.bfloat16)
    with torch.no_grad():
        m.weight.copy_(1 + 0.1 * torch.randn(H, device=DEV))
    x = (torch.randn(1, T, H, device=DEV) * 3).to(torch.bfloat16)
    xa = x.clone().requires_grad_(True)
    ya = m(xa)
    w2 = m.weight.detach().clone().requires_grad_(True)
    xb = x.clone().requires_grad_(True)
    yb = K.rmsnorm(xb, w2, 1e-6)
    _ulp_close(yb, ya, what="rmsnorm fwd")
    g = torch.randn_like(ya)
    ya.backward(g)
    yb.backward(g)
    _grad_close(xb.grad, xa.grad, "rmsnorm dx")
    _grad_close(w2.grad, m.weight.grad, "rmsnorm dw")


def test_swiglu_matches_hf():
    from verl_amd import kernels as K

    torch.manual_seed(1)
    g = (torch.randn(3, 517, 4864, device=DEV) * 2).to(torch.bfloat16)
    u = torch.randn_like(g)
    ga, ua = g.clone().requires_grad_(True), u.clone().requires_grad_(True)
    ya = F.silu(ga) * ua
    gb, ub = g.clone().requires_grad_(True), u.clone().requires_grad_(True)
    yb = K.swiglu(gb, ub)
    _ulp_close(yb, ya, what="swiglu fwd")
    d = torch.randn_like(ya)
    ya.backward(d)
    yb.backward(d)
    _grad_close(gb.grad, ga.grad, "swiglu dg")
    _grad_close(ub.grad, ua.grad, "swiglu du")


def test_rope_matches_hf():
    from transformers.models.qwen2.modeling_qwen2 import apply_rotary_pos_emb

    from verl_amd import kernels as K

    torch.manual_seed(2)
    T, Hq, Hk, D = 777, 14, 2, 64
    q = torch.randn(T, Hq, D, device=DEV).to(torch.bfloat16)
    k = torch.randn(T, Hk, D, device=DEV).to(torch.bfloat16)
    pos = torch.arange(T, device=DEV).float()
    inv = 1.0 / (1e6 ** (torch.arange(0, D, 2, device=DEV).float() / D))
    freqs = pos[:, None] * inv[None, :]
    emb = torch.cat([freqs, freqs], dim=-1)
    cos, sin = emb.cos().to(torch.bfloat16)[None], emb.sin().to(torch.bfloat16)[None]
    qa, ka = q.clone().requires_grad_(True), k.clone().requires_grad_(True)
    # HF layout [1, H, T, D]
    qe, ke = apply_rotary_pos_emb(qa.transpose(0, 1)[None], ka.transpose(0, 1)[None], cos, sin)
    qe, ke = qe[0].transpose(0, 1), ke[0].transpose(0, 1)
    qb, kb = q.clone().requires_grad_(True), k.clone().requires_grad_(True)
    qf, kf = K.rope(qb, kb, cos, sin)
    assert torch.equal(qf, qe) and torch.equal(kf, ke)  # same bf16 rounding points: bitwise
    dq, dk = torch.randn_like(qe), torch.randn_like(ke)
    (qe * dq).sum().backward(retain_graph=True)
    (ke * dk).sum().backward()
    (qf * dq).sum().backward(retain_graph=True)
    (kf * dk).sum().backward()
    _grad_close(qb.grad, qa.grad, "rope dq", rtol=1e-2)
    _grad_close(kb.grad, ka.grad, "rope dk", rtol=1e-2)


def test_patched_actor_matches_unpatched():
    from verl_amd.utils.config import actor_config
    from verl_amd.utils.model import build_qwen2
    from verl_amd.utils.synthetic import make_grpo_batch
    from verl_amd.workers.actor import DataParallelPPOActor, attention

    if not attention.varlen_available(DEV):
        pytest.skip("flash varlen unavailable")
    base = build_qwen2("tiny", device=DEV, attn_implementation="sdpa", seed=3)
    for p in base.parameters():
        p.data = p.data.to(torch.bfloat16)
    data = make_grpo_batch(n_prompts=2, n=4, prompt_len=20, response_len=30, vocab=4096, min_prompt=3,
                           dense_responses=False, min_response=5, seed=4, device=DEV)
    data.meta_info.update(micro_batch_size=4, temperature=1.0, use_dynamic_bsz=False)
    out = {}
    for fused in (False, True):
        m = copy.deepcopy(base)
        a = DataParallelPPOActor(actor_config(use_remove_padding=True, fused_model_ops=fused), m,
                                 torch.optim.SGD(m.parameters(), lr=0.0))
        lp, ent = a.compute_log_prob(data, calculate_entropy=True)
        b = data.batch
        e, lp2 = a._forward_micro_batch(b, 1.0, calculate_entropy=False)
        (lp2 * b["response_mask"]).sum().backward()
        out[fused] = (lp, ent, {n: p.grad.clone() for n, p in m.named_parameters()})
    msk = data.batch["response_mask"].bool()
    assert torch.allclose(out[True][0][msk], out[False][0][msk], atol=5e-2, rtol=2e-2)
    assert torch.allclose(out[True][1][msk], out[False][1][msk], atol=5e-2, rtol=2e-2)
    for n in out[False][2]:
        _grad_close(out[True][2][n], out[False][2][n], f"grad {n}", rtol=8e-2)
