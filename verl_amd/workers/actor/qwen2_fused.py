"""Packed (remove-padding) Qwen2 backbone forward for the actor on MI355X.

The reference runs the HF model on packed tokens with flash-attn varlen patched into HF attention
(verl/models/transformers/monkey_patch.py:50-192, dp_actor.py:104-180). Here the same math runs
through one function that owns the layer loop, so that per decoder layer the work is

  add_rmsnorm (residual add + input_layernorm, one kernel; its bwd also sums the residual grad)
  q|k|v projection as ONE GEMM (weights concatenated per call: 2 MB at H=896)
  rope_qkv   (split q/k/v into flash varlen's [T, H, D] layout + rotary, one kernel)
  flash varlen attention, o_proj GEMM
  add_rmsnorm (residual add + post_attention_layernorm)
  gate / up GEMMs, swiglu (one kernel), down GEMM

instead of the ~45 PyTorch kernels HF issues (norm chains, adds, transposes, rotary, bias
reductions x3). Forward numerics keep HF's bf16 rounding points (see csrc/model_ops.hip), so
the result matches the HF module graph to bf16 rounding (tests/test_model_ops_gpu.py).

Only bf16 Qwen2-family backbones (RMSNorm + SwiGLU MLP + rotate_half RoPE + GQA with q/k/v bias)
take this path; anything else keeps the HF forward.
"""

from __future__ import annotations

import torch
import torch.nn.functional as F

from ... import kernels as K
from . import attention


def supports(backbone: torch.nn.Module) -> bool:
    try:
        from transformers.models.qwen2 import modeling_qwen2 as m
    except ImportError:  # pragma: no cover
        return False
    if not isinstance(backbone, m.Qwen2Model):
        return False
    cfg = backbone.config
    if getattr(cfg, "hidden_act", "silu") != "silu" or getattr(cfg, "use_sliding_window", False):
        return False
    if getattr(cfg, "rope_scaling", None) not in (None, {}) and \
            (cfg.rope_scaling or {}).get("rope_type", "default") != "default":
        return False
    h = cfg.hidden_size
    if h % 8 or h > 4096:
        return False
    d = getattr(cfg, "head_dim", None) or h // cfg.num_attention_heads
    if d % 16:
        return False
    return all(p.dtype == torch.bfloat16 for p in backbone.parameters())


def _qkv_weight(attn):
    w = torch.cat([attn.q_proj.weight, attn.k_proj.weight, attn.v_proj.weight], dim=0)
    if attn.q_proj.bias is None:
        return w, None
    return w, torch.cat([attn.q_proj.bias, attn.k_proj.bias, attn.v_proj.bias], dim=0)


def _attention(attn, y, cos, sin, cu, max_len, hq, hk, d):
    T = y.shape[0]
    w, b = _qkv_weight(attn)
    qkv = F.linear(y, w, b)
    q, k, v = K.rope_qkv(qkv, cos, sin, hq, hk, d)
    out = attention.packed_attention(q, k, v, cu, max_len, scaling=attn.scaling)
    return attn.o_proj(out.reshape(T, hq * d))


def packed_forward(backbone, input_ids: torch.Tensor, position_ids: torch.Tensor, cu_seqlens: torch.Tensor,
                   max_seqlen: int) -> torch.Tensor:
    """input_ids / position_ids [T] (packed), cu_seqlens [B+1] int32 -> last hidden state [T, H] bf16
    (after the final norm), i.e. Qwen2Model(...).last_hidden_state[0] on the same packing."""
    cfg = backbone.config
    hq = cfg.num_attention_heads
    hk = cfg.num_key_value_heads
    d = getattr(cfg, "head_dim", None) or cfg.hidden_size // hq
    x = backbone.embed_tokens(input_ids)  # [T, H]
    cos, sin = backbone.rotary_emb(x.unsqueeze(0), position_ids.unsqueeze(0))  # [1, T, D] bf16
    residual = x
    layers = backbone.layers[: cfg.num_hidden_layers]
    h = None
    for i, layer in enumerate(layers):
        ln = layer.input_layernorm
        if i == 0:
            y = K.rmsnorm(residual, ln.weight, ln.variance_epsilon)
        else:
            residual, y = K.add_rmsnorm(h, residual, ln.weight, ln.variance_epsilon)
        a = _attention(layer.self_attn, y, cos, sin, cu_seqlens, max_seqlen, hq, hk, d)
        ln = layer.post_attention_layernorm
        residual, y = K.add_rmsnorm(a, residual, ln.weight, ln.variance_epsilon)
        mlp = layer.mlp
        h = mlp.down_proj(K.swiglu(mlp.gate_proj(y), mlp.up_proj(y)))
    norm = backbone.norm
    if h is None:
        return K.rmsnorm(residual, norm.weight, norm.variance_epsilon)
    _, y = K.add_rmsnorm(h, residual, norm.weight, norm.variance_epsilon)
    return y
