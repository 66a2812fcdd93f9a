"""gfx950 causal varlen flash-attention forward (attention.hip) against PyTorch-ROCm's flash
varlen kernel and an fp32 SDPA reference, plus the backward through aten's flash backward fed
with this forward's O / LSE."""

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _inputs(lens, hq=14, hk=2, d=64, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    T = int(sum(lens))
    q = torch.randn(T, hq, d, generator=g).to(torch.bfloat16).to(DEV)
    k = torch.randn(T, hk, d, generator=g).to(torch.bfloat16).to(DEV)
    v = torch.randn(T, hk, d, generator=g).to(torch.bfloat16).to(DEV)
    cu = np.zeros(len(lens) + 1, dtype=np.int64)
    np.cumsum(lens, out=cu[1:])
    return q, k, v, cu


def _restore_flash_defaults():
    from verl_amd import _lib as L

    for key, val in L.FLASH_TUNING_DEFAULTS.items():
        L.call("va_set_tuning", key, val)


def _ref_fp32(q, k, v, cu, scale):
    """Per-sequence causal SDPA in fp32 (GQA by repeat) -> O [T, Hq, D], LSE [Hq, T]."""
    hq, hk = q.shape[1], k.shape[1]
    outs, lses = [], []
    for a, b in zip(cu[:-1], cu[1:]):
        qs = q[a:b].float().transpose(0, 1)
        ks = k[a:b].float().repeat_interleave(hq // hk, dim=1).transpose(0, 1)
        vs = v[a:b].float().repeat_interleave(hq // hk, dim=1).transpose(0, 1)
        s = (qs @ ks.transpose(1, 2)) * scale
        n = b - a
        mask = torch.ones(n, n, dtype=torch.bool, device=DEV).tril()
        s = s.masked_fill(~mask, float("-inf"))
        lses.append(torch.logsumexp(s, dim=-1))
        outs.append((torch.softmax(s, dim=-1) @ vs).transpose(0, 1))
    return torch.cat(outs, 0), torch.cat(lses, 1)


@pytest.mark.parametrize("lens", [[1, 17, 128, 129, 300], [1184, 1100, 1280, 700], [64] * 9])
def test_flash_forward_matches_fp32_reference(lens):
    from verl_amd.workers.actor import attention as A

    q, k, v, cu = _inputs(lens, seed=len(lens))
    scale = 64 ** -0.5
    cu_d = torch.tensor(cu, dtype=torch.int32, device=DEV)
    blocks = torch.tensor(A.flash_block_table(cu), device=DEV)
    o = A.flash_attention(q, k, v, cu_d, int(max(lens)), blocks)
    want_o, want_lse = _ref_fp32(q, k, v, cu, scale)
    err = (o.float() - want_o).abs()
    assert err.max().item() < 2e-2, err.max().item()  # bf16 output + bf16 P
    assert err.mean().item() < 2e-3
    # LSE (aten's padded [B, Hq, max_len] layout) vs the fp32 reference
    T, mx = q.shape[0], int(max(lens))
    lse = torch.zeros(len(lens), 14, mx, device=DEV)
    from verl_amd import _lib as L
    from verl_amd import kernels as K

    o2 = torch.empty_like(q)
    L.call("va_flash_attn_fwd", K._p(q), K._p(k), K._p(v), K._p(cu_d), K._p(blocks), blocks.shape[0], T, 14, 2, 64,
           mx, scale, K._p(o2), K._p(lse), K._stream(q))
    assert torch.equal(o2, o)
    for i, (a, b) in enumerate(zip(cu[:-1], cu[1:])):
        assert (lse[i, :, : b - a] - want_lse[:, a:b]).abs().max().item() < 1e-3


@pytest.mark.parametrize("lens", [[1, 17, 128, 129, 300], [1184, 1100, 1280, 700], [64] * 9, [65, 191, 257]])
def test_flash_forward_key_block_128_equals_64(lens):
    """Forward with 128-key staged blocks equals 64-key blocks (default) bitwise: the same 64-key
    online-softmax steps in the same order."""
    from verl_amd import _lib as L
    from verl_amd import kernels as K
    from verl_amd.workers.actor import attention as A

    q, k, v, cu = _inputs(lens, seed=3 + len(lens))
    cu_d = torch.tensor(cu, dtype=torch.int32, device=DEV)
    blocks = torch.tensor(A.flash_block_table(cu), device=DEV)
    T, mx = q.shape[0], int(max(lens))
    outs = []
    try:
        for kb in (128, 64):
            L.call("va_set_tuning", L.VA_TUNE_FLASH_FWD_KB, kb)
            o = torch.empty_like(q)
            lse = torch.zeros(len(lens), 14, mx, device=DEV)
            L.call("va_flash_attn_fwd", K._p(q), K._p(k), K._p(v), K._p(cu_d), K._p(blocks), blocks.shape[0], T, 14,
                   2, 64, mx, 64 ** -0.5, K._p(o), K._p(lse), K._stream(q))
            outs.append((o, lse))
    finally:
        _restore_flash_defaults()
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("lens", [[1, 17, 128, 129, 300], [1184, 1100, 1280, 700], [64] * 9, [65, 191, 257], [3, 5]])
def test_flash_forward_dma_staging_equals_register_staging(lens):
    """VA_TUNE_FLASH_DMA bit 1 (default; K / V blocks by LDS-DMA, rows past a sequence end clamped to
    its last row instead of zeroed) equals the register-staged forward bitwise: clamped keys are masked
    to -inf and their P is 0, so the same products and sums are formed."""
    from verl_amd import _lib as L
    from verl_amd import kernels as K
    from verl_amd.workers.actor import attention as A

    q, k, v, cu = _inputs(lens, seed=11 + len(lens))
    cu_d = torch.tensor(cu, dtype=torch.int32, device=DEV)
    blocks = torch.tensor(A.flash_block_table(cu), device=DEV)
    T, mx = q.shape[0], int(max(lens))
    outs = []
    try:
        for dma in (1, 0):
            L.call("va_set_tuning", L.VA_TUNE_FLASH_DMA, dma)
            o = torch.empty_like(q)
            lse = torch.zeros(len(lens), 14, mx, device=DEV)
            L.call("va_flash_attn_fwd", K._p(q), K._p(k), K._p(v), K._p(cu_d), K._p(blocks), blocks.shape[0], T, 14,
                   2, 64, mx, 64 ** -0.5, K._p(o), K._p(lse), K._stream(q))
            outs.append((o, lse))
    finally:
        _restore_flash_defaults()
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


def test_flash_forward_matches_torch_flash_and_lse_convention():
    from verl_amd.workers.actor import attention as A

    lens = [200, 513, 1024, 77]
    q, k, v, cu = _inputs(lens, seed=5)
    cu_d = torch.tensor(cu, dtype=torch.int32, device=DEV)
    mx = int(max(lens))
    out_t, lse_t, *_ = torch.ops.aten._flash_attention_forward(q, k, v, cu_d, cu_d, mx, mx, 0.0, True,
                                                              return_debug_mask=False)
    blocks = torch.tensor(A.flash_block_table(cu), device=DEV)
    o = A.flash_attention(q, k, v, cu_d, mx, blocks)
    assert (o.float() - out_t.float()).abs().max().item() < 2e-2
    from verl_amd import _lib as L
    from verl_amd import kernels as K

    lse = torch.zeros(lse_t.shape, device=DEV, dtype=torch.float32)
    assert tuple(lse_t.shape) == (len(lens), 14, mx), lse_t.shape
    L.call("va_flash_attn_fwd", K._p(q), K._p(k), K._p(v), K._p(cu_d), K._p(blocks), blocks.shape[0], q.shape[0], 14,
           2, 64, mx, 64 ** -0.5, K._p(torch.empty_like(q)), K._p(lse), K._stream(q))
    for i, n in enumerate(lens):
        assert (lse[i, :, :n] - lse_t[i, :, :n].float()).abs().max().item() < 1e-3


@pytest.mark.parametrize("bwd", ["aten", "gfx950", "gfx950-grouped"])
@pytest.mark.parametrize("lens", [[300, 129, 1000], [1, 33, 64, 65, 128, 129, 200], [1184, 1280]])
def test_flash_backward_matches_fp32_reference(bwd, lens):
    """dQ, dK, dV of the gfx950 forward + (aten | gfx950) backward against fp32 autograd of the
    reference SDPA, and against PyTorch-ROCm's own varlen flash (fwd + bwd) at the same data."""
    from torch.nn.attention.varlen import varlen_attn

    from verl_amd.workers.actor import attention as A

    q, k, v, cu = _inputs(lens, seed=7 + len(lens))
    cu_d = torch.tensor(cu, dtype=torch.int32, device=DEV)
    mx = int(max(lens))
    g = torch.randn_like(q)
    qr, kr, vr = (t.float().clone().requires_grad_(True) for t in (q, k, v))
    want, _ = _ref_fp32(qr, kr, vr, cu, 64 ** -0.5)
    want.backward(g.float())
    qa, ka, va = (t.clone().requires_grad_(True) for t in (q, k, v))
    varlen_attn(qa, ka, va, cu_d, cu_d, mx, mx, is_causal=True).backward(g)
    qb, kb, vb = (t.clone().requires_grad_(True) for t in (q, k, v))
    blocks = torch.tensor(A.flash_block_table(cu), device=DEV)
    kblocks = torch.tensor(A.flash_key_block_table(cu), device=DEV)
    from verl_amd import _lib as L

    old = A.FLASH_BWD
    A.FLASH_BWD = bwd.split("-")[0]
    # grouped: one workgroup per key block x KV head (forced); plain gfx950: per-head partials
    L.call("va_set_tuning", L.VA_TUNE_FLASH_GROUPED_DKDV, 1 if bwd.endswith("grouped") else 0)
    try:
        A.flash_attention(qb, kb, vb, cu_d, mx, blocks, kblocks=kblocks).backward(g)
    finally:
        A.FLASH_BWD = old
        L.call("va_set_tuning", L.VA_TUNE_FLASH_GROUPED_DKDV, -1)
    for ref_t, tor, ours, what in ((qr.grad, qa.grad, qb.grad, "dq"), (kr.grad, ka.grad, kb.grad, "dk"),
                                   (vr.grad, va.grad, vb.grad, "dv")):
        r = ref_t.float()
        e_ours = ((ours.float() - r).norm() / r.norm()).item()
        e_torch = ((tor.float() - r).norm() / r.norm()).item()
        # bf16 inputs / outputs: both kernels sit at bf16 rounding of the fp32 truth
        assert e_ours < max(1.5 * e_torch, 1e-2), f"{what}: ours {e_ours:.3e} vs torch flash {e_torch:.3e}"


@pytest.mark.parametrize("grouped", [0, 1])
@pytest.mark.parametrize("lens", [[300, 129, 1000], [1, 33, 64, 65, 128, 129, 200], [1184, 1280]])
def test_flash_backward_query_tile_64_equals_32(grouped, lens):
    """dK / dV staged in 64- or 128-row query tiles (128 = default) and dQ in 128-key blocks equal
    the 32-row / 64-key stagings bitwise: the same 32-wide products in the same order (tails too)."""
    from verl_amd import _lib as L
    from verl_amd.workers.actor import attention as A

    q, k, v, cu = _inputs(lens, seed=11 + len(lens))
    cu_d = torch.tensor(cu, dtype=torch.int32, device=DEV)
    mx = int(max(lens))
    g = torch.randn_like(q)
    blocks = torch.tensor(A.flash_block_table(cu), device=DEV)
    kblocks = torch.tensor(A.flash_key_block_table(cu), device=DEV)
    grads = []
    old = A.FLASH_BWD
    A.FLASH_BWD = "gfx950"
    L.call("va_set_tuning", L.VA_TUNE_FLASH_GROUPED_DKDV, grouped)
    try:
        for qt, kblk in ((64, 128), (32, 64), (128, 128)):
            L.call("va_set_tuning", L.VA_TUNE_FLASH_DKDV_QT, qt)
            L.call("va_set_tuning", L.VA_TUNE_FLASH_DQ_KB, kblk)
            qb, kb, vb = (t.clone().requires_grad_(True) for t in (q, k, v))
            A.flash_attention(qb, kb, vb, cu_d, mx, blocks, kblocks=kblocks).backward(g)
            grads.append((qb.grad, kb.grad, vb.grad))
    finally:
        A.FLASH_BWD = old
        _restore_flash_defaults()
    for other in grads[1:]:
        for a, b in zip(grads[0], other):
            assert torch.equal(a, b)


@pytest.mark.parametrize("kblk,qt,grouped", [(64, 64, 1), (128, 128, 1), (128, 128, 0), (128, 32, 0)])
@pytest.mark.parametrize("lens", [[300, 129, 1000], [1, 33, 64, 65, 128, 129, 200], [1184, 1280], [3, 5]])
def test_flash_backward_dma_staging_equals_register_staging(kblk, qt, grouped, lens):
    """VA_TUNE_FLASH_DMA bits 2 / 4 (the dQ kernel's K / V blocks, the dK / dV kernel's Q / dO tiles by
    LDS-DMA, rows past a sequence end clamped: their P and dS are 0) and bit 1 (the forward) give
    the register-staged gradients bitwise, grouped and per-query-head dK / dV."""
    from verl_amd import _lib as L
    from verl_amd.workers.actor import attention as A

    q, k, v, cu = _inputs(lens, seed=21 + len(lens))
    cu_d = torch.tensor(cu, dtype=torch.int32, device=DEV)
    mx = int(max(lens))
    g = torch.randn_like(q)
    blocks = torch.tensor(A.flash_block_table(cu), device=DEV)
    kblocks = torch.tensor(A.flash_key_block_table(cu), device=DEV)
    grads = []
    old = A.FLASH_BWD
    A.FLASH_BWD = "gfx950"
    L.call("va_set_tuning", L.VA_TUNE_FLASH_DQ_KB, kblk)
    L.call("va_set_tuning", L.VA_TUNE_FLASH_DKDV_QT, qt)
    L.call("va_set_tuning", L.VA_TUNE_FLASH_GROUPED_DKDV, grouped)
    try:
        for dma in (7, 4, 2, 0):
            L.call("va_set_tuning", L.VA_TUNE_FLASH_DMA, dma)
            qb, kb, vb = (t.clone().requires_grad_(True) for t in (q, k, v))
            A.flash_attention(qb, kb, vb, cu_d, mx, blocks, kblocks=kblocks).backward(g)
            grads.append((qb.grad, kb.grad, vb.grad))
    finally:
        A.FLASH_BWD = old
        _restore_flash_defaults()
    for other in grads[1:]:
        for a, b in zip(grads[0], other):
            assert torch.equal(a, b)


def test_actor_with_flash_forward_matches_torch_flash():
    import copy

    from verl_amd.utils.config import actor_config
    from verl_amd.utils.model import build_qwen2
    from verl_amd.utils.synthetic import make_grpo_batch
    from verl_amd.workers.actor import DataParallelPPOActor

    base = build_qwen2("tiny", device=DEV, attn_implementation="sdpa", seed=3, hidden_size=256,
                       num_attention_heads=4, num_key_value_heads=2)  # head_dim 64
    for p in base.parameters():
        p.data = p.data.to(torch.bfloat16)
    data = make_grpo_batch(n_prompts=2, n=4, prompt_len=40, response_len=90, vocab=4096, min_prompt=3,
                           dense_responses=False, min_response=5, seed=4, device=DEV)
    data.meta_info.update(micro_batch_size=4, temperature=1.0, use_dynamic_bsz=False)
    res = {}
    for fa in (False, True):
        m = copy.deepcopy(base)
        a = DataParallelPPOActor(actor_config(use_remove_padding=True, fused_attention=fa), m,
                                 torch.optim.SGD(m.parameters(), lr=0.0))
        lp, ent = a.compute_log_prob(data, calculate_entropy=True)
        b = data.batch
        _, lp2 = a._forward_micro_batch(b, 1.0)
        (lp2 * b["response_mask"]).sum().backward()
        res[fa] = (lp, ent, {n: p.grad.clone() for n, p in m.named_parameters()})
    msk = data.batch["response_mask"].bool()
    assert torch.allclose(res[True][0][msk], res[False][0][msk], atol=5e-2, rtol=2e-2)
    for n in res[False][2]:
        a, b = res[True][2][n].float(), res[False][2][n].float()
        assert ((a - b).norm() / (b.norm() + 1e-12)) < 8e-2, n
