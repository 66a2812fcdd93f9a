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


@pytest.mark.parametrize("T,F_", [(1, 8), (3, 4864), (517, 4864), (77, 2056), (1025, 64)])
def test_swiglu_stream_matches_grid_stride(T, F_):
    """The streaming SwiGLU kernels (VA_TUNE_SWIGLU_STREAM, default) and the grid-stride ones do
    the same per-element arithmetic: bitwise equal y and merged d(gate|up), ragged tails included."""
    from verl_amd import _lib as L
    from verl_amd import kernels as K

    torch.manual_seed(T + F_)
    gu = (torch.randn(T, 2 * F_, device=DEV) * 2).to(torch.bfloat16)
    d = torch.randn(T, F_, device=DEV).to(torch.bfloat16)
    outs = []
    try:
        for v in (-1, 0):
            L.call("va_set_tuning", L.VA_TUNE_SWIGLU_STREAM, v)
            x = gu.clone().requires_grad_(True)
            y = K.swiglu_merged(x)
            y.backward(d)
            outs.append((y.detach(), x.grad))
    finally:
        L.call("va_set_tuning", L.VA_TUNE_SWIGLU_STREAM, -1)
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


def test_add_rmsnorm_matches_hf():
    """Residual add + RMSNorm (Qwen2DecoderLayer: h = residual + x; norm(h)); both outputs and the
    gradient that reaches x / residual through h and through the norm."""
    from transformers.models.qwen2.modeling_qwen2 import Qwen2RMSNorm

    from verl_amd import kernels as K

    torch.manual_seed(5)
    T, H = 1531, 896
    m = Qwen2RMSNorm(H, eps=1e-6).to(DEV).to(torch.bfloat16)
    with torch.no_grad():
        m.weight.copy_(1 + 0.1 * torch.randn(H, device=DEV))
    x = (torch.randn(T, H, device=DEV) * 2).to(torch.bfloat16)
    r = (torch.randn(T, H, device=DEV) * 4).to(torch.bfloat16)
    xa, ra = x.clone().requires_grad_(True), r.clone().requires_grad_(True)
    ha = ra + xa
    ya = m(ha)
    w2 = m.weight.detach().clone().requires_grad_(True)
    xb, rb = x.clone().requires_grad_(True), r.clone().requires_grad_(True)
    hb, yb = K.add_rmsnorm(xb, rb, w2, 1e-6)
    assert torch.equal(hb, ha)
    _ulp_close(yb, ya, what="add_rmsnorm fwd")
    gh, gy = torch.randn_like(ha), torch.randn_like(ya)
    torch.autograd.backward([ha, ya], [gh, gy])
    torch.autograd.backward([hb, yb], [gh, gy])
    _grad_close(xb.grad, xa.grad, "add_rmsnorm dx")
    _grad_close(rb.grad, ra.grad, "add_rmsnorm dres")
    _grad_close(w2.grad, m.weight.grad, "add_rmsnorm dw")


@pytest.mark.parametrize("H", [64, 896, 1536, 3584])
def test_rmsnorm_widths(H):
    """Every register-tile width (NV = 1, 2, 4, 8 vectors per lane) against the HF module."""
    from transformers.models.qwen2.modeling_qwen2 import Qwen2RMSNorm

    from verl_amd import kernels as K

    torch.manual_seed(H)
    T = 333
    m = Qwen2RMSNorm(H, eps=1e-6).to(DEV).to(torch.bfloat16)
    x = torch.randn(T, H, device=DEV).to(torch.bfloat16)
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    w2 = m.weight.detach().clone().requires_grad_(True)
    ya, yb = m(xa), K.rmsnorm(xb, w2, 1e-6)
    _ulp_close(yb, ya, what=f"rmsnorm H={H}")
    g = torch.randn_like(ya)
    ya.backward(g)
    yb.backward(g)
    _grad_close(xb.grad, xa.grad, f"rmsnorm dx H={H}")
    _grad_close(w2.grad, m.weight.grad, f"rmsnorm dw H={H}")


def test_rope_qkv_matches_hf():
    from transformers.models.qwen2.modeling_qwen2 import apply_rotary_pos_emb

    from verl_amd import kernels as K

    torch.manual_seed(2)
    T, Hq, Hk, D = 777, 14, 2, 64
    qkv = torch.randn(T, (Hq + 2 * Hk) * D, device=DEV).to(torch.bfloat16)
    pos = torch.arange(T, device=DEV).float()
    inv = 1.0 / (1e6 ** (torch.arange(0, D, 2, device=DEV).float() / D))
    freqs = pos[:, None] * inv[None, :]
    emb = torch.cat([freqs, freqs], dim=-1)
    cos, sin = emb.cos().to(torch.bfloat16)[None], emb.sin().to(torch.bfloat16)[None]
    qa_in = qkv.clone().requires_grad_(True)
    q = qa_in[:, : Hq * D].view(T, Hq, D)
    k = qa_in[:, Hq * D : (Hq + Hk) * D].view(T, Hk, D)
    v = qa_in[:, (Hq + Hk) * D :].view(T, Hk, D)
    # HF layout [1, H, T, D]
    qe, ke = apply_rotary_pos_emb(q.transpose(0, 1)[None], k.transpose(0, 1)[None], cos, sin)
    qe, ke = qe[0].transpose(0, 1), ke[0].transpose(0, 1)
    qb_in = qkv.clone().requires_grad_(True)
    qf, kf, vf = K.rope_qkv(qb_in, cos, sin, Hq, Hk, D)
    assert torch.equal(qf, qe) and torch.equal(kf, ke) and torch.equal(vf, v)  # same rounding: bitwise
    dq, dk, dv = torch.randn_like(qe), torch.randn_like(ke), torch.randn_like(v)
    torch.autograd.backward([qe, ke, v], [dq, dk, dv])
    torch.autograd.backward([qf, kf, vf], [dq, dk, dv])
    _grad_close(qb_in.grad, qa_in.grad, "rope dqkv", rtol=1e-2)


@pytest.mark.parametrize("family", ["qwen2", "llama"])
def test_patched_actor_matches_unpatched(family):
    """Fused packed backbone (gfx950 RMSNorm / SwiGLU / RoPE / flash attention, merged GEMMs) vs the
    HF forward on the same packing: log-probs, entropies and every parameter gradient. Llama covers
    BASELINE config 3's actor architecture (no q/k/v bias, untied head, Llama-3.1 rope scaling)."""
    from verl_amd.utils.config import actor_config
    from verl_amd.utils.model import build_llama, build_qwen2
    from verl_amd.utils.synthetic import make_grpo_batch
    from verl_amd.workers.actor import DataParallelPPOActor, attention

    if not attention.varlen_available(DEV):
        pytest.skip("flash varlen unavailable")
    build = {"qwen2": build_qwen2, "llama": build_llama}[family]
    base = build("tiny", device=DEV, attn_implementation="sdpa", seed=3)
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
        assert a._fused_backbone is fused, "fused packed backbone not taken"
        out[fused] = (lp, ent, {n: p.grad.clone() for n, p in m.named_parameters()})
    msk = data.batch["response_mask"].bool()
    assert torch.allclose(out[True][0][msk], out[False][0][msk], atol=5e-2, rtol=2e-2)
    assert torch.allclose(out[True][1][msk], out[False][1][msk], atol=5e-2, rtol=2e-2)
    for n in out[False][2]:
        _grad_close(out[True][2][n], out[False][2][n], f"grad {n}", rtol=8e-2)


def test_merged_linear_routes_gradients():
    """q|k|v as one GEMM over a merged buffer: output and per-parameter gradients equal the three
    separate F.linear calls."""
    from verl_amd import kernels as K
    from verl_amd.workers.actor.qwen2_fused import _merged

    torch.manual_seed(7)
    lins = [torch.nn.Linear(96, n).to(DEV).to(torch.bfloat16) for n in (96, 32, 32)]
    ref = copy.deepcopy(lins)
    x = torch.randn(500, 96, device=DEV).to(torch.bfloat16)
    owner = torch.nn.Module()
    ws, bs = [l.weight for l in lins], [l.bias for l in lins]
    w_all, b_all = _merged(owner, "w", ws), _merged(owner, "b", bs)
    assert lins[1].weight.data_ptr() == w_all.data_ptr() + 96 * 96 * 2
    y = K.merged_linear(x, w_all, b_all, ws, bs)
    y_ref = torch.cat([F.linear(x, l.weight, l.bias) for l in ref], dim=1)
    assert torch.equal(y, y_ref)
    g = torch.randn_like(y)
    y.backward(g)
    y_ref.backward(g)
    for a, b in zip(lins, ref):
        _grad_close(a.weight.grad, b.weight.grad, "merged dW", rtol=1e-2)
        _grad_close(a.bias.grad, b.bias.grad, "merged db", rtol=1e-2)


def test_fused_worker_training_tracks_master_weights():
    """Two GRPO updates through ActorWorker with bf16/fp32-master mixed precision: the fused packed
    backbone (merged q|k|v, gate|up views) and the HF forward give the same log-probs after each
    optimizer step, i.e. the fp32->bf16 copy-back lands in the merged buffers."""
    import numpy as np

    from verl_amd.trainer.ppo.core_algos import AdvantageEstimator
    from verl_amd.trainer.ppo.ray_trainer import compute_advantage
    from verl_amd.utils.config import AttrDict, actor_config
    from verl_amd.utils.model import build_qwen2
    from verl_amd.utils.synthetic import make_grpo_batch
    from verl_amd.workers.actor import attention
    from verl_amd.workers.dp_workers import ActorWorker

    if not attention.varlen_available(DEV):
        pytest.skip("flash varlen unavailable")
    base = build_qwen2("tiny", device=DEV, attn_implementation="sdpa", seed=11)
    lps = {}
    for fused in (False, True):
        cfg = AttrDict(actor=actor_config(ppo_mini_batch_size=2, ppo_micro_batch_size_per_gpu=4, use_kl_loss=True,
                                          use_remove_padding=True, fused_model_ops=fused,
                                          optim=AttrDict(lr=1e-3, weight_decay=0.01, betas=(0.9, 0.999))),
                       rollout=AttrDict(log_prob_micro_batch_size_per_gpu=8, temperature=1.0))
        w = ActorWorker(cfg, rollout_n=4).init_model(copy.deepcopy(base))
        data = make_grpo_batch(n_prompts=2, n=4, prompt_len=16, response_len=24, vocab=4096, min_prompt=3,
                               dense_responses=False, min_response=5, seed=12, device=DEV)
        data.meta_info.update(temperature=1.0)
        hist = []
        for _ in range(2):
            out = w.compute_log_prob(data)
            hist.append(out.batch["old_log_probs"].clone())
            data.batch["old_log_probs"] = out.batch["old_log_probs"]
            data.batch["ref_log_prob"] = out.batch["old_log_probs"].clone()
            compute_advantage(data, AdvantageEstimator.GRPO)
            met = w.update_actor(data).meta_info["metrics"]
            assert all(np.isfinite(v) for v in met["actor/pg_loss"])
        hist.append(w.compute_log_prob(data).batch["old_log_probs"].clone())
        assert w.actor._fused_backbone is fused
        lps[fused] = hist
    m = data.batch["response_mask"].bool()
    moved = (lps[True][2][m] - lps[True][0][m]).abs().max().item()
    assert moved > 1e-3, "weights did not change: the master copy-back missed the merged buffers"
    for a, b in zip(lps[True], lps[False]):
        assert torch.allclose(a[m], b[m], atol=5e-2, rtol=2e-2), (a[m] - b[m]).abs().max().item()


@pytest.mark.parametrize("n_out,n_in,T", [(1152, 896, 8192), (896, 4864, 8192), (896, 896, 40000),
                                          (9728, 896, 9473), (1152, 896, 77824)])
def test_splitk_weight_grad(n_out, n_in, T):
    """Split-K weight gradient (S token slices as one fp32 batched GEMM + the T % S tail, summed in
    fp32, one rounding) vs one GEMM in fp32."""
    from verl_amd import kernels as K

    torch.manual_seed(n_out)
    dy = torch.randn(T, n_out, device=DEV).to(torch.bfloat16)
    x = torch.randn(T, n_in, device=DEV).to(torch.bfloat16)
    got = K.weight_grad(dy, x)
    want = dy.float().t() @ x.float()
    _grad_close(got, want, "split-K dW", rtol=5e-3)
    base = (dy.t() @ x).float()
    assert (got.float() - want).norm() <= 1.5 * (base - want).norm() + 1e-3


@pytest.mark.parametrize("T,C", [(163840, 1152), (1000, 64), (4099, 2048), (1, 8), (0, 1152)])
def test_column_sum_matches_fp32_sum(T, C):
    """va_column_sum (the q|k|v bias gradient, kernels.column_sum): an fp32-accumulated column sum
    rounded once to bf16 — within one bf16 unit of torch's fp64 sum of the same bf16 values — on
    contiguous and row-strided inputs, deterministic run to run; zero rows give zeros."""
    from verl_amd import kernels as K

    g = torch.Generator(device=DEV).manual_seed(T + C)
    base = torch.randn(T, C + 16, device=DEV, generator=g).to(torch.bfloat16)
    for x in (base[:, :C].contiguous(), base[:, :C]):
        got = K.column_sum(x)
        want = x.double().sum(0)
        assert got.dtype == torch.bfloat16 and got.shape == (C,)
        tol = want.abs().to(torch.float32) * 2 ** -8 + 1e-3 * (T ** 0.5 + 1)
        assert torch.all((got.double() - want).abs() <= tol.double()), (got.double() - want).abs().max()
        assert torch.equal(got, K.column_sum(x))


def test_merged_linear_bias_gradient_uses_column_sum():
    """The merged q|k|v linear's bias gradient (kernels._MergedLinear) is the column sum of dY."""
    from verl_amd import kernels as K

    torch.manual_seed(0)
    x = torch.randn(300, 64, device=DEV).to(torch.bfloat16).requires_grad_(True)
    w = torch.randn(96, 64, device=DEV).to(torch.bfloat16).requires_grad_(True)
    b = torch.randn(96, device=DEV).to(torch.bfloat16).requires_grad_(True)
    y = K.merged_linear(x, w, b, [w], [b])
    dy = torch.randn_like(y)
    y.backward(dy)
    assert torch.equal(b.grad, K.column_sum(dy))
    assert (b.grad.double() - dy.double().sum(0)).abs().max().item() < 0.1


def _exact_operands(T, H, F_, ldx=None, seed=0):
    """Integer-valued x and w / 8: every partial sum of x w^T is exact in fp32, so any summation order
    gives the same projection (and the same bf16 rounding of it)."""
    g = torch.Generator(device=DEV).manual_seed(seed)
    xs = torch.randint(-2, 3, (T, ldx or H), device=DEV, generator=g).to(torch.bfloat16)
    w = (torch.randint(-3, 4, (2 * F_, H), device=DEV, generator=g).float() / 8).to(torch.bfloat16)
    return xs[:, :H], w


@pytest.mark.parametrize("T,H,F_,ldx,splits", [(1000, 896, 4864, None, None), (256, 64, 128, None, 1),
                                                (517, 256, 512, 320, 3), (3, 128, 256, None, 64),
                                                (4096, 896, 4864, None, 19)])
def test_gate_up_swiglu_bitwise_on_exact_data(T, H, F_, ldx, splits):
    """va_gate_up_swiglu == merged GEMM (hipBLASLt) + swiglu_merged, bit for bit, when the projection is
    exact: the same bf16 rounding points and per-element arithmetic; ragged token tails, a strided x,
    feature ranges per token block from 1 to the tile count."""
    from verl_amd import kernels as K

    x, w = _exact_operands(T, H, F_, ldx, seed=T + F_)
    with torch.no_grad():
        want = K.swiglu_merged(x @ w.t())
        got = K.gate_up_swiglu(x, w, splits=splits)
    assert got.shape == (T, F_)
    assert torch.equal(got, want)


@pytest.mark.parametrize("T,H,F_,ldx", [(1000, 896, 4864, None), (517, 256, 512, 320), (3, 128, 256, None)])
def test_gate_up_swiglu_save_bitwise_on_exact_data(T, H, F_, ldx):
    """va_gate_up_swiglu_save (ABI 8): y as va_gate_up_swiglu and the saved projection equal to the
    merged GEMM's bf16 output, bit for bit, on exact data (ragged tails, strided x)."""
    from verl_amd import kernels as K

    x, w = _exact_operands(T, H, F_, ldx, seed=3 * T + F_)
    with torch.no_grad():
        gu_want = x @ w.t()
        y_want = K.swiglu_merged(gu_want)
        y, gu = K._gate_up_swiglu_raw(x, w, None, save=True)
    assert torch.equal(gu, gu_want)
    assert torch.equal(y, y_want)


@pytest.mark.parametrize("defer", [0, 1])
@pytest.mark.parametrize("T,H,F_,splits", [(1000, 896, 4864, None), (517, 256, 512, 3), (3, 128, 256, 64)])
def test_gate_up_swiglu_epilogue_placement_bitwise(defer, T, H, F_, splits):
    """VA_TUNE_T256_DEFER bit 1: the tile epilogue before or after the step's operand wait writes the
    same y and projection, equal to GEMM + swiglu_merged on exact data."""
    from verl_amd import _lib as L
    from verl_amd import kernels as K

    x, w = _exact_operands(T, H, F_, None, seed=5 * T + F_)
    try:
        L.call("va_set_tuning", L.VA_TUNE_T256_DEFER, defer)
        with torch.no_grad():
            gu_want = x @ w.t()
            y_want = K.swiglu_merged(gu_want)
            y, gu = K._gate_up_swiglu_raw(x, w, splits, save=True)
            y2, _ = K._gate_up_swiglu_raw(x, w, splits, save=False)
    finally:
        L.call("va_set_tuning", L.VA_TUNE_T256_DEFER, 1)
    assert torch.equal(gu, gu_want) and torch.equal(y, y_want) and torch.equal(y2, y_want)


@pytest.mark.parametrize("T,H,F_", [(1000, 896, 4864), (300, 128, 256)])
def test_fused_mlp_train_forward_backward_bitwise_on_exact_data(T, H, F_):
    """gate_up_swiglu_train (fused_mlp_train): the activation and the gradients of x and of the gate /
    up weights equal merged_linear + swiglu_merged's bit for bit on exact data (the backward runs the
    same swiglu_bwd / dgrad / weight-gradient kernels on the same saved projection)."""
    from verl_amd import kernels as K

    x0, w0 = _exact_operands(T, H, F_, None, seed=T + 7)
    g = torch.Generator(device=DEV).manual_seed(T)
    dy = (torch.randint(-2, 3, (T, F_), device=DEV, generator=g).float() / 4).to(torch.bfloat16)
    res = {}
    for fused in (False, True):
        x = x0.clone().requires_grad_(True)
        w_all = w0.clone()
        gate = torch.nn.Parameter(w_all[:F_])
        up = torch.nn.Parameter(w_all[F_:])
        gate.data, up.data = w_all[:F_], w_all[F_:]  # views into the merged buffer, as qwen2_fused._merged
        if fused:
            y = K.gate_up_swiglu_train(x, w_all, [gate, up])
        else:
            y = K.swiglu_merged(K.merged_linear(x, w_all, None, [gate, up]))
        y.backward(dy)
        res[fused] = (y.detach(), x.grad, gate.grad, up.grad)
    for a, b, what in zip(res[True], res[False], ("y", "dx", "d_gate", "d_up")):
        assert torch.equal(a, b), what


def _qkv_case(T, H, hq, hk, seed, bias=True):
    """Exact operands for the fused q|k|v: integer x, w / 8, bias / 8 (the projection and bias sum are
    exact in fp32), and real rotary tables of packed positions."""
    g = torch.Generator(device=DEV).manual_seed(seed)
    nf = (hq + 2 * hk) * 64
    x = torch.randint(-2, 3, (T, H), device=DEV, generator=g).to(torch.bfloat16)
    w = (torch.randint(-3, 4, (nf, H), device=DEV, generator=g).float() / 8).to(torch.bfloat16)
    b = (torch.randint(-4, 5, (nf,), device=DEV, generator=g).float() / 8).to(torch.bfloat16) if bias else None
    pos = torch.randint(0, 4096, (T,), device=DEV, generator=g).float()
    inv = 1.0 / (1e6 ** (torch.arange(0, 64, 2, device=DEV).float() / 64))
    fr = pos[:, None] * inv[None]
    emb = torch.cat([fr, fr], -1)
    return x, w, b, emb.cos().to(torch.bfloat16)[None], emb.sin().to(torch.bfloat16)[None]


@pytest.mark.parametrize("defer", [1, 5])  # VA_TUNE_T256_DEFER bit 4: the epilogue after the operand wait
@pytest.mark.parametrize("T,H,hq,hk,bias", [(1000, 896, 14, 2, True), (300, 128, 4, 2, True), (37, 64, 2, 1, False),
                                            (2048, 896, 14, 2, True)])
def test_qkv_rope_bitwise_on_exact_data(defer, T, H, hq, hk, bias):
    """va_qkv_rope (ABI 9) == merged q|k|v GEMM with bias (hipBLASLt) + rope_qkv, bit for bit, on exact
    projections: q / k rotated, v passed through, ragged token tails, a last tile half past the heads."""
    from verl_amd import _lib as L
    from verl_amd import kernels as K

    x, w, b, cos, sin = _qkv_case(T, H, hq, hk, seed=T + hq)
    try:
        L.call("va_set_tuning", L.VA_TUNE_T256_DEFER, defer)
        with torch.no_grad():
            want = K.rope_qkv(torch.nn.functional.linear(x, w, b), cos, sin, hq, hk, 64)
            got = K.qkv_rope(x, w, b, cos, sin, hq, hk, 64, [w], [b] if bias else None)
    finally:
        L.call("va_set_tuning", L.VA_TUNE_T256_DEFER, 1)
    for a, e, what in zip(got, want, "qkv"):
        assert torch.equal(a, e), what


def test_qkv_rope_gradients_equal_the_unfused_path():
    """Under autograd the fused q|k|v gives the unfused path's gradients of x, the q/k/v weights and
    biases bit for bit on exact data (the backward runs the same rope_qkv_bwd / dgrad / weight and
    bias-gradient kernels)."""
    from verl_amd import kernels as K

    T, H, hq, hk = 512, 128, 4, 2
    x0, w0, b0, cos, sin = _qkv_case(T, H, hq, hk, seed=5)
    g = torch.Generator(device=DEV).manual_seed(9)
    dq, dk, dv = ((torch.randint(-2, 3, (T, n, 64), device=DEV, generator=g).float() / 4).to(torch.bfloat16)
                  for n in (hq, hk, hk))
    sizes = [hq * 64, hk * 64, hk * 64]
    res = {}
    for fused in (False, True):
        x = x0.clone().requires_grad_(True)
        w_all, b_all = w0.clone(), b0.clone()
        ws = [torch.nn.Parameter(t) for t in torch.split(w_all, sizes)]
        bs = [torch.nn.Parameter(t) for t in torch.split(b_all, sizes)]
        for p_, t in zip(ws + bs, list(torch.split(w_all, sizes)) + list(torch.split(b_all, sizes))):
            p_.data = t
        if fused:
            q, k, v = K.qkv_rope(x, w_all, b_all, cos, sin, hq, hk, 64, ws, bs)
        else:
            q, k, v = K.rope_qkv(K.merged_linear(x, w_all, b_all, ws, bs), cos, sin, hq, hk, 64)
        torch.autograd.backward([q, k, v], [dq, dk, dv])
        res[fused] = [q.detach(), k.detach(), v.detach(), x.grad] + [p_.grad for p_ in ws + bs]
    for i, (a, e) in enumerate(zip(res[True], res[False])):
        assert torch.equal(a, e), i


def test_gate_up_swiglu_random_vs_fp32():
    """Random operands: within bf16 rounding of silu(g) * u from an fp32 GEMM (tolerance: 2 bf16 ulp on
    all but 1e-3 of the elements, i.e. the product's own rounding points)."""
    from verl_amd import kernels as K

    torch.manual_seed(11)
    T, H, F_ = 3000, 896, 4864
    x = torch.randn(T, H, device=DEV).to(torch.bfloat16)
    w = (torch.randn(2 * F_, H, device=DEV) * 0.05).to(torch.bfloat16)
    with torch.no_grad():
        gu = x.float() @ w.float().t()
        ref = F.silu(gu[:, :F_].to(torch.bfloat16).float()).to(torch.bfloat16).float() * gu[:, F_:].to(torch.bfloat16).float()
        got = K.gate_up_swiglu(x, w)
        unfused = K.swiglu_merged(x @ w.t())
    _ulp_close(got, ref, n_ulp=4, what="gate_up_swiglu vs fp32")
    _ulp_close(got, unfused, n_ulp=4, what="gate_up_swiglu vs unfused")


def test_gate_up_swiglu_contract():
    from verl_amd import kernels as K

    x = torch.randn(64, 128, device=DEV).to(torch.bfloat16)
    w = torch.randn(2 * 256, 128, device=DEV).to(torch.bfloat16)
    with torch.no_grad():
        assert K.gate_up_swiglu(x[:0], w).shape == (0, 256)
        with pytest.raises(ValueError, match="unsupported"):
            K.gate_up_swiglu(x, w[: 2 * 192])  # F % 128 != 0
    with pytest.raises(RuntimeError, match="forward-only"):
        K.gate_up_swiglu(x.requires_grad_(True), w)
    assert not K.gate_up_swiglu_supported(x[:, :96], w[:, :96])


@pytest.mark.parametrize("family", ["qwen2", "llama"])
def test_fused_mlp_no_grad_pass(family):
    """fused_mlp_no_grad: compute_log_prob's packed forward runs va_gate_up_swiglu (and only there:
    the update pass keeps the merged GEMM + swiglu for its backward); log-probs match the unfused
    no-grad pass to bf16 rounding."""
    from verl_amd import kernels as K
    from verl_amd.utils.config import actor_config
    from verl_amd.utils.model import build_llama, build_qwen2
    from verl_amd.utils.synthetic import make_grpo_batch
    from verl_amd.workers.actor import DataParallelPPOActor, attention

    if not attention.varlen_available(DEV):
        pytest.skip("flash varlen unavailable")
    if family == "qwen2":
        base = build_qwen2("tiny", device=DEV, attn_implementation="sdpa", seed=5, intermediate_size=384)
    else:
        base = build_llama("tiny", device=DEV, attn_implementation="sdpa", seed=5)
    for p in base.parameters():
        p.data = p.data.to(torch.bfloat16)
    data = make_grpo_batch(n_prompts=2, n=4, prompt_len=20, response_len=30, vocab=4096, min_prompt=3,
                           dense_responses=False, min_response=5, seed=6, device=DEV)
    data.meta_info.update(micro_batch_size=4, temperature=1.0, use_dynamic_bsz=False)
    calls = []
    orig = K.gate_up_swiglu

    def spy(*a, **k):
        calls.append(1)
        return orig(*a, **k)

    out = {}
    try:
        K.gate_up_swiglu = spy
        for fused in (False, True):
            m = copy.deepcopy(base)
            a = DataParallelPPOActor(actor_config(use_remove_padding=True, fused_mlp_no_grad=fused), m,
                                     torch.optim.SGD(m.parameters(), lr=0.0))
            n0 = len(calls)
            lp, ent = a.compute_log_prob(data, calculate_entropy=True)
            n_nograd = len(calls) - n0
            e, lp2 = a._forward_micro_batch(data.batch, 1.0, calculate_entropy=False)
            (lp2 * data.batch["response_mask"]).sum().backward()
            assert len(calls) - n0 == n_nograd, "the fused MLP ran under autograd"
            assert (n_nograd > 0) == fused, n_nograd
            out[fused] = (lp, ent)
    finally:
        K.gate_up_swiglu = orig
    msk = data.batch["response_mask"].bool()
    assert torch.allclose(out[True][0][msk], out[False][0][msk], atol=3e-2, rtol=2e-2)
    assert torch.allclose(out[True][1][msk], out[False][1][msk], atol=3e-2, rtol=2e-2)
