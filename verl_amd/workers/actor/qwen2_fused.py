"""Per-instance patch of an HF Qwen2 backbone for the packed (remove-padding) actor path.

The reference patches HF attention for flash-attn varlen + Ulysses (verl/models/transformers/
monkey_patch.py:50-192). Here the patch serves MI355X launch efficiency: for bf16 weights it
replaces, module instance by module instance,

  Qwen2RMSNorm.forward  -> one fused kernel fwd, one bwd (+ column-sum for dw)   (~8+10 ops before)
  Qwen2MLP.forward      -> gate/up GEMMs + one fused SwiGLU kernel + down GEMM    (2+3 ops before)
  Qwen2Attention.forward-> q/k/v GEMMs written as [T, H, D] views, one fused RoPE kernel that also
                           produces flash varlen's layout (no transposes / contiguous copies),
                           varlen attention, o GEMM                                (~16 ops before)

Forward numerics keep HF's bf16 rounding points (see verl_amd/csrc/model_ops.hip). Other
architectures are left untouched.
"""

from __future__ import annotations

import types

import torch

from ... import kernels as K
from . import attention


def _norm_forward(self, hidden_states):
    return K.rmsnorm(hidden_states, self.weight, self.variance_epsilon)


def _mlp_forward(self, x):
    return self.down_proj(K.swiglu(self.gate_proj(x), self.up_proj(x)))


def _attn_forward(self, hidden_states, position_embeddings, attention_mask=None, past_key_values=None, **kwargs):
    cu = kwargs.get("cu_seq_lens_q")
    mx = kwargs.get("max_length_q")
    if cu is None or hidden_states.shape[0] != 1:
        raise RuntimeError("fused Qwen2 attention serves the packed varlen path (batch 1 + cu_seq_lens_q)")
    x = hidden_states[0]
    T = x.shape[0]
    D = self.head_dim
    q = self.q_proj(x).view(T, -1, D)
    k = self.k_proj(x).view(T, -1, D)
    v = self.v_proj(x).view(T, -1, D)
    cos, sin = position_embeddings
    q, k = K.rope(q, k, cos, sin)
    out = attention.packed_attention(q, k, v, cu, mx, scaling=self.scaling)
    out = self.o_proj(out.reshape(T, -1))
    return out.unsqueeze(0), None


def patch_qwen2(model: torch.nn.Module) -> int:
    """Patch every Qwen2 RMSNorm / MLP / Attention instance in ``model`` whose weights are bf16.
    Returns the number of patched modules (0 for other architectures)."""
    try:
        from transformers.models.qwen2 import modeling_qwen2 as m
    except ImportError:  # pragma: no cover
        return 0
    n = 0
    for mod in model.modules():
        if isinstance(mod, m.Qwen2RMSNorm) and mod.weight.dtype == torch.bfloat16:
            mod.forward = types.MethodType(_norm_forward, mod)
            n += 1
        elif isinstance(mod, m.Qwen2MLP) and mod.gate_proj.weight.dtype == torch.bfloat16 \
                and mod.config.hidden_act == "silu":
            mod.forward = types.MethodType(_mlp_forward, mod)
            n += 1
        elif isinstance(mod, m.Qwen2Attention) and mod.q_proj.weight.dtype == torch.bfloat16:
            mod.forward = types.MethodType(_attn_forward, mod)
            n += 1
    return n
