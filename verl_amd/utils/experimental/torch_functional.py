"""Drop-in for verl/utils/experimental/torch_functional.py (FusedLinearForPPO: the reference's
chunked-torch fused lm_head backend, `use_fused_kernels` with impl_backend "torch",
dense_common.py:71-129): the same module and call

    log_probs, entropy = FusedLinearForPPO(chunk_size)(hidden_states, vocab_weights, input_ids, temperature)

on the gfx950 fused kernels instead of chunk-by-chunk torch ops. Semantics kept from the reference
(:20-75): logits = (hidden @ W^T) / T in the inputs' dtype (bf16: two roundings — the fused kernel's
default mode), log-softmax / entropy in fp32, outputs cast back to the inputs' dtype and shaped like
input_ids ([T] or [B, S]). The backward's dlogits are rounded once after the division by T (the
reference rounds, then divides in bf16: the same bits at T = 1). ``chunk_size`` is accepted and
unused (the kernel holds no [chunk, V] logits at all).
"""

from __future__ import annotations

from typing import Optional

import torch

from ... import kernels as K


class FusedLinearForPPOFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, hidden_states, vocab_weights, input_ids, temperature: float = 1.0, chunk_size: int = 512):
        orig_ndim = hidden_states.ndim
        assert orig_ndim in (2, 3), f"Invalid hidden_states shape, received {hidden_states.shape}"
        if orig_ndim == 3:
            assert input_ids.ndim == 2, f"input_ids shape doesn't match, {hidden_states.shape} {input_ids.shape}"
        h = hidden_states.flatten(0, 1) if orig_ndim == 3 else hidden_states
        ids = input_ids.flatten(0, 1) if orig_ndim == 3 else input_ids
        with torch.enable_grad():
            hd = h.detach().requires_grad_(hidden_states.requires_grad)
            wd = vocab_weights.detach().requires_grad_(vocab_weights.requires_grad)
            lp, ent = K.linear_logprob_entropy(hd, wd, ids, float(temperature))
        ctx.inner = (hd, wd, lp, ent)
        ctx.orig_shape = hidden_states.shape
        ctx.out_shape = input_ids.shape
        dt = hidden_states.dtype
        return lp.to(dt).view(input_ids.shape), ent.to(dt).view(input_ids.shape)

    @staticmethod
    def backward(ctx, dlog_probs: Optional[torch.Tensor], dentropy: Optional[torch.Tensor]):
        assert dlog_probs is not None or dentropy is not None
        hd, wd, lp, ent = ctx.inner
        outs, grads = [], []
        for o, g in ((lp, dlog_probs), (ent, dentropy)):
            if g is not None:
                outs.append(o)
                grads.append(g.reshape(-1).float())
        inputs = [t for t in (hd, wd) if t.requires_grad]
        got = iter(torch.autograd.grad(outs, inputs, grads) if inputs else ())
        dh = next(got).view(ctx.orig_shape) if hd.requires_grad else None
        dw = next(got) if wd.requires_grad else None
        ctx.inner = None
        return dh, dw, None, None, None


class FusedLinearForPPO(torch.nn.Module):
    def __init__(self, chunk_size: int = 512):
        super().__init__()
        self.chunk_size = chunk_size

    def forward(self, hidden_states: torch.FloatTensor, vocab_weights: torch.FloatTensor,
                input_ids: torch.LongTensor, temperature: float = 1.0) -> tuple[torch.FloatTensor, torch.FloatTensor]:
        input_ids = input_ids.to(torch.int64)
        return FusedLinearForPPOFunction.apply(hidden_states, vocab_weights, input_ids, temperature, self.chunk_size)
