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


def varlen_available(device) -> bool:
    """True when PyTorch-ROCm's flash varlen kernel runs on this device."""
    try:
        q = torch.randn(24, 4, 64, device=device, dtype=torch.bfloat16)
        cu = torch.tensor([0, 10, 24], device=device, dtype=torch.int32)
        _varlen(q, q, q, cu, 14)
        return True
    except Exception:
        return False
