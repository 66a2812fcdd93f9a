"""Packed (remove-padding) Qwen2 backbone forward for the actor on MI355X.

The reference runs the HF model on packed tokens with flash-attn varlen patched into HF attention
(verl/models/transformers/monkey_patch.py:50-192, dp_actor.py:104-180). Here the same math runs
through one function that owns the layer loop, so that per decoder layer the work is

  add_rmsnorm (residual add + input_layernorm, one kernel; its bwd also sums the residual grad)
  q|k|v projection as ONE GEMM (+ one wgrad GEMM and one bias reduction in backward)
  rope_qkv   (split q/k/v into flash varlen's [T, H, D] layout + rotary, one kernel)
  flash varlen attention, o_proj GEMM
  add_rmsnorm (residual add + post_attention_layernorm)
  gate|up as ONE GEMM, swiglu on the merged output (one kernel), down GEMM

instead of the ~45 PyTorch kernels HF issues (norm chains, adds, transposes, rotary, bias
reductions x3). Forward numerics keep HF's bf16 rounding points (see csrc/model_ops.hip), so
the result matches the HF module graph to bf16 rounding (tests/test_model_ops_gpu.py).

Merging is done in memory, not in the module tree: on first use the q/k/v (and gate/up) weight
and bias Parameters of each layer are re-pointed (``param.data``) to row blocks of one buffer, so
the GEMM reads the merged matrix with no per-call concatenation while optimizers, state dicts and
the fp32-master copy-back keep addressing the original Parameters.

Only bf16 Qwen2-family backbones (RMSNorm + SwiGLU MLP + rotate_half RoPE + GQA with q/k/v bias)
take this path; anything else keeps the HF forward.
"""

from __future__ import annotations

import torch

from ... import kernels as K
from . import attention


def _decoder_families():
    """HF decoder stacks with the Qwen2 layer structure (RMSNorm, q/k/v/o projections with optional
    biases, rotate_half RoPE from the model's own rotary_emb, GQA, gate/up/down SiLU MLP): Qwen2 /
    Qwen2.5 and Llama (incl. Llama-3's rope scaling: cos / sin come from the model's rotary_emb)."""
    fams = []
    try:
        from transformers.models.qwen2 import modeling_qwen2

        fams.append(modeling_qwen2.Qwen2Model)
    except ImportError:  # pragma: no cover
        pass
    try:
        from transformers.models.llama import modeling_llama

        fams.append(modeling_llama.LlamaModel)
    except ImportError:  # pragma: no cover
        pass
    return tuple(fams)


def supports(backbone: torch.nn.Module) -> bool:
    fams = _decoder_families()
    if not fams or not isinstance(backbone, fams):
        return False
    cfg = backbone.config
    if getattr(cfg, "hidden_act", "silu") != "silu" or getattr(cfg, "use_sliding_window", False):
        return False
    rope = (getattr(cfg, "rope_scaling", None) or {})
    if rope.get("rope_type", rope.get("type", "default")) in ("mrope", "longrope"):
        return False  # multimodal / per-position factor tables: keep the HF forward
    h = cfg.hidden_size
    if h % 8 or h > 4096:
        return False
    d = getattr(cfg, "head_dim", None) or h // cfg.num_attention_heads
    if d % 16:
        return False
    return all(p.dtype == torch.bfloat16 for p in backbone.parameters())


def _merged(module, key: str, params: list):
    """Row-concatenated buffer whose row blocks are ``params`` (re-pointing them on first use or
    whenever one of them was re-allocated, e.g. by a dtype change)."""
    cache = module.__dict__.setdefault("_va_merged", {})
    ent = cache.get(key)
    if ent is not None:
        buf, ptrs = ent
        if all(p.data_ptr() == q for p, q in zip(params, ptrs)) and buf.dtype == params[0].dtype:
            return buf
    with torch.no_grad():
        buf = torch.cat([p.data.reshape(p.shape[0], -1) for p in params], dim=0)
        if params[0].dim() == 1:
            buf = buf.reshape(-1)
        off = 0
        for p in params:
            p.data = buf[off : off + p.shape[0]].view(p.shape)
            off += p.shape[0]
    cache[key] = (buf, [p.data_ptr() for p in params])
    return buf


def _merged_linear(module, key: str, x, linears: list):
    ws = [lin.weight for lin in linears]
    w_all = _merged(module, key + ".w", ws)
    if linears[0].bias is None:
        return K.merged_linear(x, w_all, None, ws)
    bs = [lin.bias for lin in linears]
    b_all = _merged(module, key + ".b", bs)
    return K.merged_linear(x, w_all, b_all, ws, bs)


def _attention(attn, y, cos, sin, cu, max_len, hq, hk, d, attn_blocks=None, attn_kblocks=None):
    T = y.shape[0]
    qkv = _merged_linear(attn, "qkv", y, [attn.q_proj, attn.k_proj, attn.v_proj])
    q, k, v = K.rope_qkv(qkv, cos, sin, hq, hk, d)
    if attn_blocks is not None and attention.flash_supported(q, k):
        out = attention.flash_attention(q, k, v, cu, max_len, attn_blocks, scaling=attn.scaling, kblocks=attn_kblocks)
    else:
        out = attention.packed_attention(q, k, v, cu, max_len, scaling=attn.scaling)
    o = attn.o_proj
    if o.bias is None:
        return K.linear(out.reshape(T, hq * d), o.weight)
    return o(out.reshape(T, hq * d))


def packed_forward(backbone, input_ids: torch.Tensor, position_ids: torch.Tensor, cu_seqlens: torch.Tensor,
                   max_seqlen: int, attn_blocks: torch.Tensor = None, attn_kblocks: torch.Tensor = None) -> torch.Tensor:
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
        a = _attention(layer.self_attn, y, cos, sin, cu_seqlens, max_seqlen, hq, hk, d, attn_blocks, attn_kblocks)
        ln = layer.post_attention_layernorm
        residual, y = K.add_rmsnorm(a, residual, ln.weight, ln.variance_epsilon)
        mlp = layer.mlp
        gu = _merged_linear(mlp, "gate_up", y, [mlp.gate_proj, mlp.up_proj])
        dp = mlp.down_proj
        a = K.swiglu_merged(gu)
        h = K.linear(a, dp.weight) if dp.bias is None else dp(a)
    norm = backbone.norm
    if h is None:
        return K.rmsnorm(residual, norm.weight, norm.variance_epsilon)
    _, y = K.add_rmsnorm(h, residual, norm.weight, norm.variance_epsilon)
    return y
