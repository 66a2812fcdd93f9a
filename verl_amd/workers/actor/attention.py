"""Packed variable-length attention for HF decoder models on MI355X.

The reference removes padding and runs flash-attn varlen over (1, total_nnz) packed tokens
(dp_actor.py:109-174, monkey_patch.py). Here the same packing feeds PyTorch-ROCm's flash
varlen kernel through transformers' AttentionInterface, so the HF model code is unchanged:
  * ``register()`` adds the attention function "verl_amd_varlen" and an always-None mask
    function, so no [nnz x nnz] mask is ever materialised;
  * the actor passes cu_seq_lens / max_length as forward kwargs (FlashAttentionKwargs).
"""

from __future__ import annotations

import torch

_NAME = "verl_amd_varlen"
_registered = False
_gqa_native: bool | None = None


def _varlen(q, k, v, cu, mx):
    from torch.nn.attention.varlen import varlen_attn

    return varlen_attn(q, k, v, cu, cu, mx, mx, is_causal=True)


def packed_attention(q, k, v, cu, mx, scaling=None):
    """Causal flash varlen attention on packed [T, H, D] tensors (GQA: Hk divides Hq)."""
    global _gqa_native
    if scaling is not None and abs(scaling - q.shape[-1] ** -0.5) > 1e-12:
        q = q * (scaling / q.shape[-1] ** -0.5)
    hq, hk = q.shape[1], k.shape[1]
    if hq != hk:
        if _gqa_native is None:
            try:
                out = _varlen(q, k, v, cu, mx)
                _gqa_native = True
                return out
            except Exception:
                _gqa_native = False
        if not _gqa_native:
            k = k.repeat_interleave(hq // hk, dim=1)
            v = v.repeat_interleave(hq // hk, dim=1)
    return _varlen(q, k, v, cu, mx)


# ------------------------------------------------------------------ gfx950 flash forward
FLASH_QB = 128  # query rows per workgroup of va_flash_attn_fwd


def _blocks(cu_host, blk: int):
    """(sequence, first row) of every ``blk``-row block of the packed sequences, in sequence order
    (host-side, vectorized: it runs on the step's critical path before the first kernel)."""
    import numpy as np

    lens = np.diff(np.asarray(cu_host, dtype=np.int64))
    counts = (lens + blk - 1) // blk
    seqs = np.repeat(np.arange(len(lens)), counts)
    first = np.repeat(np.cumsum(counts) - counts, counts)
    return seqs, (np.arange(len(seqs), dtype=np.int64) - first) * blk


def flash_block_table(cu_host) -> "np.ndarray":
    """(sequence, first query row) of every 128-row query block, heaviest (latest) blocks first so
    the causal tail of long sequences does not end the launch on a few workgroups."""
    import numpy as np

    seqs, starts = _blocks(cu_host, FLASH_QB)
    order = np.lexsort((seqs, -starts))  # by start descending, then sequence
    return np.stack([seqs[order], starts[order]], axis=1).astype(np.int32)


FLASH_KB = 128  # keys per workgroup of the dK / dV kernel


def flash_key_block_table(cu_host) -> "np.ndarray":
    """(sequence, first key) of every 128-key block, earliest (heaviest under the causal mask)
    blocks first."""
    import numpy as np

    seqs, starts = _blocks(cu_host, FLASH_KB)
    order = np.lexsort((seqs, starts))
    return np.stack([seqs[order], starts[order]], axis=1).astype(np.int32)


# backward implementation: "gfx950" (va_flash_attn_bwd) or "aten" (AOTriton flash backward)
FLASH_BWD = "gfx950"


class _FlashVarlen(torch.autograd.Function):
    """Forward: va_flash_attn_fwd (gfx950 MFMA kernel). Backward: va_flash_attn_bwd (delta, dK/dV,
    dQ kernels), or aten._flash_attention_backward fed with this forward's O and LSE."""

    @staticmethod
    def forward(ctx, q, k, v, cu, blocks, max_len, scale, kblocks=None):
        from ... import _lib as L
        from ... import kernels as K

        T, hq, d = q.shape
        hk = k.shape[1]
        o = torch.empty_like(q)
        # aten's varlen flash LSE layout [B, Hq, max_len]; padded rows stay 0 (finite)
        lse = torch.zeros(cu.shape[0] - 1, hq, int(max_len), dtype=torch.float32, device=q.device)
        L.call("va_flash_attn_fwd", K._p(q), K._p(k), K._p(v), K._p(cu), K._p(blocks), blocks.shape[0], T, hq, hk, d,
               int(max_len), float(scale), K._p(o), K._p(lse), K._stream(q))
        ctx.save_for_backward(q, k, v, o, lse, cu, blocks, kblocks if kblocks is not None else blocks)
        ctx.has_kblocks = kblocks is not None
        ctx.max_len = int(max_len)
        ctx.scale = float(scale)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, cu, blocks, kblocks = ctx.saved_tensors
        do = do.contiguous()
        if FLASH_BWD == "gfx950" and ctx.has_kblocks:
            from ... import _lib as L
            from ... import kernels as K

            T, hq, d = q.shape
            hk = k.shape[1]
            dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
            delta = torch.zeros_like(lse)
            partial = torch.empty(2 * hq * T * d, dtype=torch.float32, device=q.device)
            L.call("va_flash_attn_bwd", K._p(q), K._p(k), K._p(v), K._p(o), K._p(do), K._p(lse), K._p(cu),
                   K._p(blocks), blocks.shape[0], K._p(kblocks), kblocks.shape[0], T, hq, hk, d, ctx.max_len,
                   ctx.scale, K._p(delta), K._p(partial), K._p(dq), K._p(dk), K._p(dv), K._stream(q))
            return dq, dk, dv, None, None, None, None, None
        rng = torch.zeros(2, dtype=torch.uint64, device=q.device)
        unused = torch.empty(0, device=q.device)
        dq, dk, dv = torch.ops.aten._flash_attention_backward(
            do, q, k, v, o, lse, cu, cu, ctx.max_len, ctx.max_len, 0.0, True, rng, unused, scale=ctx.scale)
        return dq, dk, dv, None, None, None, None, None


def flash_attention(q, k, v, cu, max_len, blocks, scaling=None, kblocks=None):
    """Causal varlen attention on packed [T, H, 64] bf16 tensors with the gfx950 kernels.
    ``blocks`` = device int32 [n, 2] from flash_block_table; ``kblocks`` from
    flash_key_block_table enables the gfx950 backward (else aten's)."""
    scale = q.shape[-1] ** -0.5 if scaling is None else scaling
    return _FlashVarlen.apply(q.contiguous(), k.contiguous(), v.contiguous(), cu, blocks, max_len, scale, kblocks)


def flash_supported(q, k) -> bool:
    return (q.is_cuda and q.dtype == torch.bfloat16 and k.dtype == torch.bfloat16 and q.shape[-1] == 64
            and q.shape[1] % k.shape[1] == 0)


def varlen_attention_forward(module, query, key, value, attention_mask, scaling=None, dropout=0.0, **kwargs):
    """AttentionInterface entry: query [1, Hq, nnz, D], key/value [1, Hkv, nnz, D] ->
    ([1, nnz, Hq, D], None)."""
    cu = kwargs.get("cu_seq_lens_q")
    mx = kwargs.get("max_length_q")
    if cu is None:
        raise RuntimeError("verl_amd_varlen attention needs cu_seq_lens_q / max_length_q kwargs")
    assert query.shape[0] == 1, "packed varlen attention expects batch 1"
    # RoPE's fp32 cos/sin promote q/k to fp32 under autocast; flash runs in the autocast dtype
    if torch.is_autocast_enabled("cuda"):
        dt = torch.get_autocast_dtype("cuda")
    else:
        dt = value.dtype if value.dtype in (torch.float16, torch.bfloat16) else torch.bfloat16
    q = query[0].transpose(0, 1).to(dt).contiguous()
    k = key[0].transpose(0, 1).to(dt).contiguous()
    v = value[0].transpose(0, 1).to(dt).contiguous()
    out = packed_attention(q, k, v, cu, mx, scaling)
    return out.unsqueeze(0), None


def _no_mask(*args, **kwargs):
    return None


def register() -> str:
    global _registered
    if not _registered:
        from transformers import AttentionInterface, AttentionMaskInterface

        AttentionInterface.register(_NAME, varlen_attention_forward)
        AttentionMaskInterface.register(_NAME, _no_mask)
        _registered = True
    return _NAME


def use_packed_attention(model, backbone) -> None:
    """Route the decoder's HF attention through the packed varlen function. For Qwen2-VL only the
    language model's config is switched: its vision tower runs full (non-causal) attention over
    image patches with its own implementation."""
    name = register()
    from .qwen2_fused import text_backbone

    stack = text_backbone(backbone)
    if stack is not backbone:
        stack.config._attn_implementation = name
    elif hasattr(model, "set_attn_implementation"):
        model.set_attn_implementation(name)
    else:
        model.config._attn_implementation = name


def varlen_available(device) -> bool:
    """True when PyTorch-ROCm's flash varlen kernel runs on this device."""
    try:
        q = torch.randn(24, 4, 64, device=device, dtype=torch.bfloat16)
        cu = torch.tensor([0, 10, 24], device=device, dtype=torch.int32)
        _varlen(q, q, q, cu, 14)
        return True
    except Exception:
        return False
