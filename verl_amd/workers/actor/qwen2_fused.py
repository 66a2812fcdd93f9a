"""Packed (remove-padding) Qwen2 backbone forward for the actor on MI355X.

The reference runs the HF model on packed tokens with flash-attn varlen patched into HF attention
(verl/models/transformers/monkey_patch.py:50-192, dp_actor.py:104-180). Here the same math runs
through one function that owns the layer loop, so that per decoder layer the work is

  add_rmsnorm (residual add + input_layernorm, one kernel; its bwd also sums the residual grad)
  q|k|v projection as ONE GEMM (+ one wgrad GEMM and one bias reduction in backward)
  rope_qkv   (split q/k/v into flash varlen's [T, H, D] layout + rotary, one kernel)
  flash varlen attention, o_proj GEMM
  add_rmsnorm (residual add + post_attention_layernorm)
  gate|up as ONE GEMM, swiglu on the merged output (one kernel), down GEMM — in a no-grad forward
  (the old-logp pass) gate|up + swiglu are ONE kernel (va_gate_up_swiglu: no [T, 2F] projection)

instead of the ~45 PyTorch kernels HF issues (norm chains, adds, transposes, rotary, bias
reductions x3). Forward numerics keep HF's bf16 rounding points (see csrc/model_ops.hip), so
the result matches the HF module graph to bf16 rounding (tests/test_model_ops_gpu.py).

Merging is done in memory, not in the module tree: on first use the q/k/v (and gate/up) weight
and bias Parameters of each layer are re-pointed (``param.data``) to row blocks of one buffer, so
the GEMM reads the merged matrix with no per-call concatenation while optimizers, state dicts and
the fp32-master copy-back keep addressing the original Parameters.

Only bf16 Qwen2-family backbones (RMSNorm + SwiGLU MLP + rotate_half RoPE + GQA with q/k/v bias)
take this path; anything else keeps the HF forward. Qwen2-VL's language model (BASELINE config 4)
is the same decoder with multimodal RoPE: its packed position ids are [3, T] (temporal, height,
width; dp_actor.py:106-121) and the rotary cos / sin of each channel section come from one of the
three rows (transformers' apply_multimodal_rotary_pos_emb), after which the same rope_qkv kernel
applies. Image / video embeddings come from the model's own vision tower (HF, outside SURVEY §8)
and are scattered over the placeholder tokens of the packed sequence, as the HF model does.
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
    vl = _qwen2_vl_text_model()
    if vl is not None:
        fams.append(vl)
    return tuple(fams)


def _qwen2_vl_text_model():
    try:
        from transformers.models.qwen2_vl import modeling_qwen2_vl

        return modeling_qwen2_vl.Qwen2VLTextModel
    except ImportError:  # pragma: no cover
        return None


def text_backbone(backbone: torch.nn.Module) -> torch.nn.Module:
    """The decoder stack of an actor / critic backbone: Qwen2-VL's Qwen2VLModel keeps it as
    ``language_model`` beside the vision tower ``visual``; text models are their own stack."""
    lm = getattr(backbone, "language_model", None)
    return lm if lm is not None and hasattr(backbone, "visual") else backbone


def mrope_section(stack: torch.nn.Module):
    """Channel sections (temporal, height, width) of a multimodal-RoPE decoder stack, else None."""
    vl = _qwen2_vl_text_model()
    if vl is None or not isinstance(stack, vl):
        return None
    rope = getattr(stack.config, "rope_parameters", None) or getattr(stack.config, "rope_scaling", None) or {}
    sec = rope.get("mrope_section")
    return list(sec) if sec else None


def supports(backbone: torch.nn.Module) -> bool:
    stack = text_backbone(backbone)
    fams = _decoder_families()
    if not fams or not isinstance(stack, fams):
        return False
    cfg = stack.config
    if getattr(cfg, "hidden_act", "silu") != "silu" or getattr(cfg, "use_sliding_window", False):
        return False
    h = cfg.hidden_size
    if h % 8 or h > 4096:
        return False
    d = getattr(cfg, "head_dim", None) or h // cfg.num_attention_heads
    if d % 16:
        return False
    sec = mrope_section(stack)
    if sec is not None:
        if sum(sec) != d // 2:
            return False
    else:
        rope = (getattr(cfg, "rope_scaling", None) or {})
        if rope.get("rope_type", rope.get("type", "default")) in ("mrope", "longrope"):
            return False  # per-position factor tables / unknown multimodal layouts: keep the HF forward
    return all(p.dtype == torch.bfloat16 for p in stack.parameters())


def rotary(stack: torch.nn.Module, x: torch.Tensor, position_ids: torch.Tensor):
    """cos / sin [1, T, D] of packed positions: [T] for 1-D RoPE; [3, T] (or [T], replicated as
    the HF text model does for text-only input) for multimodal RoPE, where channel section i of
    the doubled section list takes row i % 3 (apply_multimodal_rotary_pos_emb)."""
    sec = mrope_section(stack)
    if sec is None:
        return stack.rotary_emb(x.unsqueeze(0), position_ids.unsqueeze(0))
    if position_ids.dim() == 1:
        position_ids = position_ids.expand(3, -1)
    cos, sin = stack.rotary_emb(x.unsqueeze(0), position_ids.unsqueeze(1))  # [3, 1, T, D]
    parts = sec * 2
    cos = torch.cat([c[i % 3] for i, c in enumerate(cos.split(parts, dim=-1))], dim=-1)
    sin = torch.cat([s_[i % 3] for i, s_ in enumerate(sin.split(parts, dim=-1))], dim=-1)
    return cos, sin


def input_embeddings(backbone: torch.nn.Module, input_ids: torch.Tensor, multi_modal_inputs: list = None):
    """Token embeddings of a packed sequence [T] -> [T, H]. For Qwen2-VL with multi_modal_inputs
    (one dict per row: pixel_values / image_grid_thw, pixel_values_videos / video_grid_thw,
    concatenated in row order as dp_actor.py:94-98), the vision tower's outputs replace the image /
    video placeholder tokens in order (Qwen2VLModel.forward). The packing keeps row order and token
    order, so the placeholders meet the images in the same order as in the padded batch."""
    stack = text_backbone(backbone)
    x = stack.embed_tokens(input_ids)
    if not multi_modal_inputs:
        return x
    if stack is backbone:
        raise NotImplementedError("multi_modal_inputs given to a text-only backbone")
    mm = {k: torch.cat([d[k] for d in multi_modal_inputs], dim=0).to(input_ids.device) for k in multi_modal_inputs[0]}
    cfg = backbone.config
    for pix, grid, tok, fn in (("pixel_values", "image_grid_thw", "image_token_id", "get_image_features"),
                               ("pixel_values_videos", "video_grid_thw", "video_token_id", "get_video_features")):
        if pix not in mm:
            continue
        out = getattr(backbone, fn)(mm[pix], mm[grid])
        emb = getattr(out, "pooler_output", out)
        emb = torch.cat(list(emb), dim=0) if isinstance(emb, (list, tuple)) else emb
        sel = input_ids == getattr(cfg, tok)
        n = int(sel.sum())
        if n != emb.shape[0]:
            raise ValueError(f"{pix}: {emb.shape[0]} vision embeddings for {n} placeholder tokens")
        x = x.masked_scatter(sel.unsqueeze(-1), emb.to(x.dtype))
    return x


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


def _qkv(attn, y, cos, sin, hq, hk, d, fuse: bool):
    """q, k, v [T, H, D] after RoPE: the merged q|k|v GEMM + the RoPE kernel, or (``fuse``) one kernel
    with the bias and RoPE in the GEMM's epilogue (va_qkv_rope)."""
    lins = [attn.q_proj, attn.k_proj, attn.v_proj]
    if fuse:
        ws = [lin.weight for lin in lins]
        w_all = _merged(attn, "qkv.w", ws)
        bs = [lin.bias for lin in lins] if lins[0].bias is not None else None
        b_all = _merged(attn, "qkv.b", bs) if bs else None
        if K.qkv_rope_supported(y, w_all, b_all, cos, d, hq, hk, sin):
            return K.qkv_rope(y, w_all, b_all, cos, sin, hq, hk, d, ws, bs)
    qkv = _merged_linear(attn, "qkv", y, lins)
    return K.rope_qkv(qkv, cos, sin, hq, hk, d)


def _attention(attn, y, cos, sin, cu, max_len, hq, hk, d, attn_blocks=None, attn_kblocks=None, fuse_qkv=False):
    T = y.shape[0]
    q, k, v = _qkv(attn, y, cos, sin, hq, hk, d, fuse_qkv)
    if attn_blocks is not None and attention.flash_supported(q, k):
        out = attention.flash_attention(q, k, v, cu, max_len, attn_blocks, scaling=attn.scaling, kblocks=attn_kblocks)
    else:
        out = attention.packed_attention(q, k, v, cu, max_len, scaling=attn.scaling)
    o = attn.o_proj
    if o.bias is None:
        return K.linear(out.reshape(T, hq * d), o.weight)
    return o(out.reshape(T, hq * d))


def _mlp_activation(mlp, y, fuse: bool, fuse_train: bool = False):
    """silu(gate_proj(y)) * up_proj(y): one fused kernel when the shapes allow (and the projections
    carry no bias) — in the no-grad forward (``fuse``: no projection written) and, with
    ``fuse_train``, under autograd (the kernel also writes the projection for the backward) — else
    the merged GEMM + the SwiGLU kernel."""
    lins = [mlp.gate_proj, mlp.up_proj]
    training = torch.is_grad_enabled() and (y.requires_grad or lins[0].weight.requires_grad)
    if (fuse_train if training else fuse) and lins[0].bias is None:
        ws = [lin.weight for lin in lins]
        w_all = _merged(mlp, "gate_up.w", ws)
        if K.gate_up_swiglu_supported(y, w_all):
            return K.gate_up_swiglu_train(y, w_all, ws) if training else K.gate_up_swiglu(y, w_all)
    return K.swiglu_merged(_merged_linear(mlp, "gate_up", y, lins))


def packed_forward(backbone, input_ids: torch.Tensor, position_ids: torch.Tensor, cu_seqlens: torch.Tensor,
                   max_seqlen: int, attn_blocks: torch.Tensor = None, attn_kblocks: torch.Tensor = None,
                   multi_modal_inputs: list = None, fuse_mlp: bool = False,
                   fuse_mlp_train: bool = False, fuse_qkv: bool = False) -> torch.Tensor:
    """input_ids [T] and position_ids [T] (or [3, T], mrope) packed, cu_seqlens [B+1] int32 -> last
    hidden state [T, H] bf16 (after the final norm), i.e. Qwen2Model(...).last_hidden_state[0] on
    the same packing. ``fuse_mlp``: outside autograd, gate|up + SwiGLU run as one kernel
    (va_gate_up_swiglu; its GEMM sums in its own order, so the hidden states match the unfused
    forward to bf16 rounding, not bitwise). ``fuse_mlp_train``: under autograd, the same kernel also
    writes the projection for the SwiGLU backward (va_gate_up_swiglu_save). ``fuse_qkv``: the q|k|v
    GEMM, its bias and RoPE as one kernel (va_qkv_rope), in both passes."""
    stack = text_backbone(backbone)
    cfg = stack.config
    hq = cfg.num_attention_heads
    hk = cfg.num_key_value_heads
    d = getattr(cfg, "head_dim", None) or cfg.hidden_size // hq
    x = input_embeddings(backbone, input_ids, multi_modal_inputs)  # [T, H]
    cos, sin = rotary(stack, x, position_ids)  # [1, T, D] bf16
    residual = x
    fuse_mlp = bool(fuse_mlp) and not torch.is_grad_enabled()
    layers = stack.layers[: cfg.num_hidden_layers]
    h = None
    for i, layer in enumerate(layers):
        ln = layer.input_layernorm
        if i == 0:
            y = K.rmsnorm(residual, ln.weight, ln.variance_epsilon)
        else:
            residual, y = K.add_rmsnorm(h, residual, ln.weight, ln.variance_epsilon)
        a = _attention(layer.self_attn, y, cos, sin, cu_seqlens, max_seqlen, hq, hk, d, attn_blocks, attn_kblocks,
                       fuse_qkv=fuse_qkv)
        ln = layer.post_attention_layernorm
        residual, y = K.add_rmsnorm(a, residual, ln.weight, ln.variance_epsilon)
        mlp = layer.mlp
        dp = mlp.down_proj
        a = _mlp_activation(mlp, y, fuse_mlp, fuse_mlp_train)
        h = K.linear(a, dp.weight) if dp.bias is None else dp(a)
    norm = stack.norm
    if h is None:
        return K.rmsnorm(residual, norm.weight, norm.variance_epsilon)
    _, y = K.add_rmsnorm(h, residual, norm.weight, norm.variance_epsilon)
    return y
