"""Drop-in for verl/utils/kernel/linear_cross_entropy.py:40-117, the reference's fused lm_head GEMM +
log-softmax gather + entropy (its Triton kernels, kernels.py:120-1553; `use_fused_kernels` with
impl_backend "triton", dense_common.py:133-193 / monkey_patch.py:148-192): the same call

    logprobs, entropy = linear_cross_entropy(hidden, weight, labels, temperature, reduction, dist_process_group)

on the gfx950 fused kernels (va_linear_logprob_fwd; va_linear_logprob_bwd per vocab range, the
reference's _Split_Dlogits_N loop): no [N, V] logits or dlogits in HBM. As in the reference,

* hidden [..., H] and labels [...] are flattened; logprobs / entropy come back flat [N] (fp32);
* the logits are fp32 (no bf16 rounding: the kernels' VA_LOGITS_F32 mode), divided by temperature;
* reduction "none" returns per-token log-probs, "sum" / "mean" their sum / mean (EntropyReductionEnum,
  kernels.py:60-70); entropy is always per token;
* dist_process_group: vocab tensor parallelism. ``weight`` is this rank's shard of rows
  [rank V_s, (rank + 1) V_s) of the vocabulary, labels are global ids. The forward merges the shards'
  row statistics with one MAX and one SUM all-reduce (the reference's epilogue_tp / tp_update,
  kernels.py:349-468, 609-660); the backward writes this shard's dlogits against the merged lse and
  entropy and returns the shard's d_weight and its PARTIAL d_hidden (the reference leaves that
  all-reduce to the caller: tests/utils/test_linear_cross_entropy_tp.py:409-422).
"""

from __future__ import annotations

import types

import torch
import torch.distributed as dist

from ... import kernels as K
from . import kernels as _cfg

# EntropyReductionEnum (kernels.py:60-70)
REDUCTIONS = {"none": 0, "sum": 1, "mean": 2}


def _reduction_code(reduction: str) -> int:
    r = REDUCTIONS.get(reduction.lower())
    if r is None:
        raise ValueError(f"Invalid reduction: {reduction}")
    return r


def tp_merge(labels, vocab_offset: int, vocab_shard: int, vocab_total: int, logp_l, ent_l, lse_l,
             all_reduce_max, all_reduce_sum, label_logit_l=None):
    """Merge one vocabulary shard's per-row (logp, entropy, lse) — the shard's own softmax, labels
    shifted into the shard — into the whole vocabulary's, given the group's MAX / SUM all-reduces:
      m = max_r lse_r, A = sum_r e^{lse_r - m}, B = sum_r e^{lse_r - m} (lse_r - H_r),
      lse = m + ln A, H = lse - B / A, logp = x[label] - lse,
    x[label] contributed by the shard that holds it. Labels: -100 (ignore_index) gives 0, other ids
    outside the vocabulary NaN, as va_linear_logprob_fwd. x[label] is the raw label logit of the shard
    that holds it (``label_logit_l``, the kernel's own value), all-reduced as the reference's epilogue_tp
    does; without it, rebuilt as logp_r + lse_r in fp32 (~ulp(lse_r) of rounding)."""
    in_shard = (labels >= vocab_offset) & (labels < vocab_offset + vocab_shard)
    xl = logp_l + lse_l if label_logit_l is None else label_logit_l
    xlab = torch.where(in_shard, xl, torch.zeros_like(lse_l))
    m = lse_l.clone()
    all_reduce_max(m)
    s = torch.exp(lse_l - m)
    packed = torch.stack([s, s * (lse_l - ent_l), xlab])
    all_reduce_sum(packed)
    lse = m + torch.log(packed[0])
    ent = lse - packed[1] / packed[0]
    valid = (labels >= 0) & (labels < vocab_total)
    other = torch.where(labels == -100, torch.zeros_like(lse), torch.full_like(lse, float("nan")))
    logp = torch.where(valid, packed[2] - lse, other)
    return logp, ent, lse


class LinearCrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, hidden, weight, labels, temperature=1.0, reduction="none", dist_process_group=None):
        assert isinstance(temperature, float), f"temperature must be a float, but got {type(temperature)}"
        assert isinstance(reduction, str), f"reduction must be a str, but got {type(reduction)}"
        red = _reduction_code(reduction)
        K._require_device(hidden, weight, labels)
        K._bf16_only(hidden, weight)
        shape = hidden.shape
        h = hidden.reshape(-1, shape[-1])
        if h.stride(-1) != 1 or h.stride(0) % 8 or h.data_ptr() % 16:
            h = h.contiguous()
        w = weight if weight.stride(-1) == 1 and weight.stride(0) % 8 == 0 else weight.contiguous()
        if w.dim() != 2 or w.shape[1] != h.shape[1]:
            raise ValueError(f"linear_cross_entropy: hidden {tuple(shape)} vs weight {tuple(weight.shape)}")
        lab = labels.reshape(-1).long().contiguous()
        if lab.shape[0] != h.shape[0]:
            raise ValueError(f"labels ({lab.shape[0]}) do not match hidden rows ({h.shape[0]})")
        vs = w.shape[0]
        if dist_process_group is None:
            off, total = 0, vs
            logp, ent, lse = K._linear_logprob_fwd_raw(h, w, lab, temperature, fp32_logits=True)
        else:
            if vs % 4:
                raise ValueError(f"linear_cross_entropy: a vocabulary shard must be a multiple of 4 rows, got {vs}")
            rank, world = dist.get_rank(dist_process_group), dist.get_world_size(dist_process_group)
            off, total = rank * vs, world * vs
            logp_l, ent_l, lse_l, xl = K._linear_logprob_fwd_raw(h, w, lab - off, temperature, fp32_logits=True,
                                                                 with_label_logit=True)
            logp, ent, lse = tp_merge(
                lab, off, vs, total, logp_l, ent_l, lse_l,
                lambda t: dist.all_reduce(t, op=dist.ReduceOp.MAX, group=dist_process_group),
                lambda t: dist.all_reduce(t, op=dist.ReduceOp.SUM, group=dist_process_group), label_logit_l=xl)
        ctx.save_for_backward(h, w, lab, lse, ent)
        ctx.hidden_shape = shape
        ctx.reduction = red
        ctx.temperature = temperature
        ctx.vocab_offset, ctx.vocab_total = off, total
        if red == 0:
            return logp, ent
        total_lp = logp.sum()
        return (total_lp if red == 1 else total_lp / max(lab.shape[0], 1)), ent

    @staticmethod
    def backward(ctx, dlogprobs, dentropy):
        h, w, lab, lse, ent = ctx.saved_tensors
        N = h.shape[0]
        need_h, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        if N == 0:
            return (torch.zeros(ctx.hidden_shape, dtype=h.dtype, device=h.device) if need_h else None,
                    torch.zeros_like(w) if need_w else None, None, None, None, None)
        g1 = None
        if dlogprobs is not None:
            g1 = dlogprobs.float()
            if ctx.reduction != 0:  # a scalar: every row's log-prob enters with the same weight
                g1 = (g1 / N if ctx.reduction == 2 else g1).reshape(1).expand(N).contiguous()
            else:
                g1 = g1.contiguous()
        g2 = None if dentropy is None else dentropy.float().contiguous()
        if w.shape[0] % 4:  # the composition path (whole vocabulary only)
            kctx = types.SimpleNamespace(needs_input_grad=(need_h, need_w), temperature=ctx.temperature,
                                         fp32_logits=True)
            d_hidden, d_weight = K._LinearLogprob._compose_backward(kctx, h, w, lab, lse, ent, g1, g2)
        else:
            # the dlogits range width of the configured backward method (kernels.set_backward_method)
            kctx = types.SimpleNamespace(needs_input_grad=(need_h, need_w), temperature=ctx.temperature,
                                         fp32_logits=True, vocab_offset=ctx.vocab_offset,
                                         vocab_total=ctx.vocab_total,
                                         vocab_per_split=_cfg.backward_vocab_per_split(
                                             w.shape[0], K._LinearLogprob.VOCAB_PER_SPLIT))
            d_hidden, d_weight = K._LinearLogprob._vocab_split_backward(kctx, h, w, lab, lse, ent, g1, g2)
        if d_hidden is not None:
            d_hidden = d_hidden.view(ctx.hidden_shape)
        return d_hidden, d_weight, None, None, None, None


linear_cross_entropy = LinearCrossEntropy.apply
