"""Drop-in mirror of verl/utils/torch_functional.py for the actor-update hot path.

Same function names, argument meaning and error texts as the reference; the arithmetic runs
in the gfx950 kernels (verl_amd.kernels). Inputs must live on the HIP device.
"""

from __future__ import annotations

import torch
import torch.distributed

from .. import _lib as L
from .. import kernels as K

__all__ = [
    "gather_from_labels", "logprobs_from_logits", "logprobs_from_logits_v2", "logprobs_and_entropy_from_logits",
    "entropy_from_logits", "entropy_from_logits_with_chunking", "masked_sum", "masked_mean", "masked_var",
    "masked_whiten", "clip_by_value", "get_response_mask", "distributed_mean_max_min_std",
    "distributed_masked_mean", "allgather_dict_tensors", "broadcast_dict_tensor",
    "get_constant_schedule_with_warmup", "get_cosine_schedule_with_warmup", "get_wsd_schedule_with_warmup",
    "logprobs_from_logits_naive", "logprobs_from_logits_flash_attn", "log_probs_from_logits_response",
    "log_probs_from_logits_response_rmpad", "log_probs_from_logits_all_rmpad", "post_process_logits",
    "compute_grad_norm", "get_unpad_data", "remove_pad_token", "pad_sequence_to_length", "pad_2d_list_to_length",
]


def gather_from_labels(data, label):
    """torch_functional.py:49-61."""
    return torch.gather(data, -1, label.unsqueeze(-1)).squeeze(-1)


def logprobs_from_logits(logits, labels, inplace_backward=True):
    """torch_functional.py:64-92: log p(label) over the last dim, fp32 result.

    One fused HBM pass (va_logprob_entropy_fwd); the backward is a second pass that writes
    dlogits — into the logits buffer when ``inplace_backward`` (flash-attn semantics).
    """
    logp, _ = K.logprob_entropy(logits, labels, 1.0, inplace_backward)
    return logp


def logprobs_from_logits_naive(logits, labels):
    """torch_functional.py:110-113 (log_softmax + gather): the same values from the one-pass kernel."""
    return logprobs_from_logits(logits, labels, inplace_backward=False)


def logprobs_from_logits_flash_attn(logits, labels, inplace_backward=True):
    """torch_functional.py:95-100 (flash-attn's cross_entropy_loss with inplace_backward): the
    kernel pair this module's logprobs_from_logits runs."""
    return logprobs_from_logits(logits, labels, inplace_backward=inplace_backward)


def _unpad_indices(attention_mask):
    return torch.nonzero(attention_mask.flatten(), as_tuple=False).flatten()


def _pad_rows(values, indices, batch: int, seqlen: int):
    """flash_attn.bert_padding.pad_input for a [nnz] vector: zeros at the padded positions."""
    out = torch.zeros(batch * seqlen, dtype=values.dtype, device=values.device)
    out[indices] = values
    return out.view(batch, seqlen)


def log_probs_from_logits_response(input_ids, logits, response_length):
    """torch_functional.py:422-435: log-probs of the response tokens from the full [B, S, V] logits
    (logits at position t predict token t + 1)."""
    response_logits = logits[:, -response_length - 1 : -1]
    response = input_ids[:, -response_length:]
    return logprobs_from_logits(logits=response_logits, labels=response)


def log_probs_from_logits_response_rmpad(input_ids, attention_mask, logits_rmpad, response_length):
    """torch_functional.py:438-462: log-probs from remove-padding logits [nnz, V] of the padded
    input_ids [B, S]: labels are the packed ids rolled by one (torch.roll over the whole packed
    stream, as the reference), scattered back to [B, S] and cut to the response."""
    batch_size, seqlen = input_ids.shape
    indices = _unpad_indices(attention_mask)
    ids_rmpad = input_ids.flatten()[indices]
    rolled = torch.roll(ids_rmpad, shifts=-1, dims=0)
    full = logprobs_from_logits(logits=logits_rmpad, labels=rolled)
    return _pad_rows(full, indices, batch_size, seqlen)[:, -response_length - 1 : -1]


def log_probs_from_logits_all_rmpad(input_ids_rmpad, logits_rmpad, indices, batch_size, seqlen, response_length):
    """torch_functional.py:465-490: as log_probs_from_logits_response_rmpad with the packed ids
    [1, nnz] and their unpad indices given."""
    ids = input_ids_rmpad.transpose(0, 1).squeeze(-1)
    rolled = torch.roll(ids, shifts=-1, dims=0)
    full = logprobs_from_logits(logits=logits_rmpad, labels=rolled)
    return _pad_rows(full, indices, batch_size, seqlen)[:, -response_length - 1 : -1]


def post_process_logits(input_ids, logits, temperature, top_k, top_p):
    """torch_functional.py:493-500: logits.div_(temperature) in place (top-k / top-p are disabled
    there too)."""
    if temperature != 1.0:
        logits = logits.div_(temperature)
    return logits


def logprobs_from_logits_v2(logits, labels):
    """torch_functional.py:116-133 (memory-efficient variant): same result, one pass."""
    return logprobs_from_logits(logits, labels, inplace_backward=False)


def logprobs_and_entropy_from_logits(logits, labels, temperature: float = 1.0, inplace_backward: bool = False):
    """Fused dp_actor.py:182-201: ``logits.div_(T)`` + logprobs_from_logits + entropy_from_logits
    in one read of the logits (the reference reads them twice or three times)."""
    return K.logprob_entropy(logits, labels, temperature, inplace_backward)


def _entropy(logits):
    V = logits.shape[-1]
    dummy = torch.zeros(logits.shape[:-1], dtype=torch.int64, device=logits.device)
    _, ent = K.logprob_entropy(logits, dummy, 1.0, False)
    del V
    return ent


def entropy_from_logits(logits: torch.Tensor):
    """torch_functional.py:145-149: logsumexp(x) - sum(softmax(x) * x), fp32 math."""
    return _entropy(logits)


def entropy_from_logits_with_chunking(logits: torch.Tensor, chunk_size: int = 2048):
    """torch_functional.py:152-160 (fp32 upcast per chunk): the kernel streams rows anyway."""
    return _entropy(logits)


def clip_by_value(x, tensor_min, tensor_max):
    """torch_functional.py:136-142."""
    return torch.max(torch.min(x, tensor_max), tensor_min)


def masked_sum(values, mask, axis=None):
    """torch_functional.py:163-168."""
    if axis is None:
        return K.masked_aggregate(values, mask, L.VA_REDUCE_MASKED_SUM)
    return (torch.where(mask.bool(), values, 0.0) * mask).sum(axis=axis)


def masked_mean(values, mask, axis=None):
    """torch_functional.py:171-185: sum(where(m, x, 0) * m) / (sum(m) + 1e-8)."""
    if axis is None:
        return K.masked_aggregate(values, mask, L.VA_AGG_TOKEN_MEAN)
    nd = values.dim()
    ax = axis if isinstance(axis, int) else None
    if ax is not None and ax % nd == nd - 1:
        return K.masked_aggregate(values, mask.expand_as(values), L.VA_REDUCE_ROW_MASKED_MEAN)
    if ax is not None:
        v = values.movedim(ax, -1).contiguous()
        m = mask.expand_as(values).movedim(ax, -1).contiguous()
        return K.masked_aggregate(v, m, L.VA_REDUCE_ROW_MASKED_MEAN)
    s = (torch.where(mask.bool(), values, 0.0) * mask).sum(axis=axis)
    return s / (mask.sum(axis=axis) + 1e-8)


def _merged_var(merged: torch.Tensor, unbiased: bool) -> torch.Tensor:
    n, s, m2 = merged[0], merged[1], merged[2]
    mean = s / (n + 1e-8)
    mu = torch.where(n > 0, s / n.clamp(min=1e-300), torch.zeros_like(n))
    var = (m2 + n * (mu - mean) ** 2) / (n + 1e-8)
    if unbiased:
        nv = float(n.item())
        if nv == 0:
            raise ValueError("At least one element in the mask has to be 1.")
        if nv == 1:
            raise ValueError("The sum of the mask is one, which can cause a division by zero.")
        var = var * (n / (n - 1))
    return var.float()


def masked_var(values, mask, unbiased=True):
    """torch_functional.py:188-203 (ValueError when the mask sums to 0 or 1 and unbiased)."""
    _, merged = K.whiten_stats(values, mask)
    return _merged_var(merged, unbiased)


def masked_whiten(values, mask, shift_mean=True):
    """torch_functional.py:206-223: (x - mean) * rsqrt(var + 1e-8), stats over the mask."""
    stats, _ = K.whiten_stats(values, mask)
    K._raise_whiten_flag(stats)
    out = K.whiten_apply(values, mask, stats)
    if not shift_mean:
        out += stats[0]
    return out


def get_response_mask(response_id: torch.Tensor, eos_token=2, dtype=torch.int64):
    """torch_functional.py:226-246: 1 up to and including the first EOS, 0 after."""
    eos = torch.isin(response_id, torch.tensor(eos_token, device=response_id.device)).int()
    return (eos.cumsum(dim=1) - eos).eq(0).to(dtype)


def distributed_mean_max_min_std(local_tensor, compute_max=True, compute_min=True, compute_std=True):
    """torch_functional.py:709-749: global stats with one SUM all-reduce of (sum, count)."""
    dev = local_tensor.device
    packed = torch.stack([local_tensor.sum().float(), torch.tensor(float(local_tensor.numel()), device=dev)])
    torch.distributed.all_reduce(packed, op=torch.distributed.ReduceOp.SUM)
    mean = packed[0] / packed[1]
    gmax = gmin = gstd = None
    if compute_max:
        gmax = local_tensor.max().clone()
        torch.distributed.all_reduce(gmax, op=torch.distributed.ReduceOp.MAX)
    if compute_min:
        gmin = local_tensor.min().clone()
        torch.distributed.all_reduce(gmin, op=torch.distributed.ReduceOp.MIN)
    if compute_std:
        sq = torch.sum((local_tensor - mean) ** 2)
        torch.distributed.all_reduce(sq, op=torch.distributed.ReduceOp.SUM)
        gstd = torch.sqrt(sq / (packed[1] - 1))
    return mean, gmax, gmin, gstd


def distributed_masked_mean(local_tensor, local_mask):
    """torch_functional.py:752-771: one all-reduce of (sum(x*m), sum(m))."""
    packed = torch.stack([(local_tensor * local_mask).sum().float(), local_mask.sum().float()])
    torch.distributed.all_reduce(packed, op=torch.distributed.ReduceOp.SUM)
    return packed[0] / packed[1]


def compute_grad_norm(model: torch.nn.Module):
    """torch_functional.py:249-254: the SUM OF SQUARES of all gradients (no square root), a host
    float. One device reduction over all gradients instead of a host sync per parameter."""
    grads = [p.grad.detach() for p in model.parameters() if p.grad is not None]
    if not grads:
        return 0
    sq = torch._foreach_norm(grads, 2.0)
    return float(torch.sum(torch.stack([g.double() for g in sq]) ** 2).item())


def get_unpad_data(attention_mask):
    """torch_functional.py:629-638: (indices of the valid tokens, cu_seqlens int32, max seqlen)."""
    seqlens = attention_mask.sum(dim=-1, dtype=torch.int32)
    indices = _unpad_indices(attention_mask)
    cu = torch.nn.functional.pad(torch.cumsum(seqlens, dim=0, dtype=torch.int32), (1, 0))
    return indices, cu, int(seqlens.max().item())


def remove_pad_token(input_ids: torch.Tensor, attention_mask: torch.Tensor):
    """torch_functional.py:407-419: per row, the last mask.sum() ids (left padding removed), as lists."""
    return [ids[len(ids) - int(mask.sum()):].cpu().numpy().tolist()
            for ids, mask in zip(input_ids, attention_mask, strict=True)]


def pad_sequence_to_length(tensors, max_seq_len, pad_token_id, left_pad=False):
    """torch_functional.py:318-328: pad the last dim to max_seq_len (unchanged when already longer)."""
    if tensors.shape[-1] >= max_seq_len:
        return tensors
    n = max_seq_len - tensors.shape[-1]
    return torch.nn.functional.pad(tensors, (n, 0) if left_pad else (0, n), "constant", pad_token_id)


def pad_2d_list_to_length(response, pad_token_id, max_length=None):
    """torch_functional.py:307-315: a ragged 2-D list right-padded into a tensor."""
    longest = max(len(r) for r in response)
    target = max_length if max_length is not None and max_length > longest else longest
    return torch.tensor([tuple(r) + (pad_token_id,) * (target - len(r)) for r in response])


def broadcast_dict_tensor(tensors, src, group):
    for key in sorted(tensors.keys()):
        torch.distributed.broadcast(tensors[key], src=src, group=group, async_op=False)


def allgather_dict_tensors(tensors, size, group, dim=0):
    """torch_functional.py:266-297 (dict form)."""
    out = {}
    for key in sorted(tensors.keys()):
        val = tensors[key].contiguous()
        parts = [torch.empty_like(val) for _ in range(size)]
        torch.distributed.all_gather(parts, val, group=group, async_op=False)
        out[key] = torch.cat(parts, dim=dim)
    return out


# ------------------------------------------------------------------ LR schedules (host)
def get_cosine_schedule_with_warmup(optimizer, num_warmup_steps: int, num_training_steps: int,
                                    min_lr_ratio: float = 0.0, num_cycles: float = 0.5, last_epoch: int = -1):
    """torch_functional.py:509-550: a linear ramp from min_lr_ratio to 1 over the warmup steps,
    then 0.5 (1 + min) + 0.5 (1 - min) cos(2 pi cycles progress), floored at min_lr_ratio."""
    import math

    from torch.optim.lr_scheduler import LambdaLR

    min_lr_ratio = 0.0 if min_lr_ratio is None else min_lr_ratio
    assert 0.0 <= min_lr_ratio <= 1.0
    half_span, mid = (1.0 - min_lr_ratio) * 0.5, (1.0 + min_lr_ratio) * 0.5
    warm, total = int(num_warmup_steps), int(num_training_steps)

    def factor(step: int) -> float:
        if step < warm:
            return min_lr_ratio + (1.0 - min_lr_ratio) * (float(step) / float(max(1, warm)))
        progress = float(step - warm) / float(max(1, total - warm))
        return max(min_lr_ratio, math.cos(math.pi * float(num_cycles) * 2.0 * progress) * half_span + mid)

    return LambdaLR(optimizer, factor, last_epoch)


def get_constant_schedule_with_warmup(optimizer, num_warmup_steps: int, last_epoch: int = -1):
    """torch_functional.py:553-575: step / warmup during the warmup steps, then 1."""
    from torch.optim.lr_scheduler import LambdaLR

    warm = num_warmup_steps

    def factor(step: int) -> float:
        return float(step) / float(max(1.0, warm)) if step < warm else 1.0

    return LambdaLR(optimizer, factor, last_epoch)


def get_wsd_schedule_with_warmup(optimizer, num_warmup_steps: int, num_training_steps: int,
                                 min_lr_ratio: float = 0.0, num_cycles: float = 0.5, last_epoch: int = -1,
                                 stable_ratio: float = 0.9):
    """torch_functional.py:641-694: warmup (linear from 0), stable (1), then cosine decay to
    min_lr_ratio over the last (1 - stable_ratio) of the post-warmup steps, min_lr_ratio after."""
    import math

    from torch.optim.lr_scheduler import LambdaLR

    remaining = max(0, num_training_steps - num_warmup_steps)
    stable = int(remaining * stable_ratio)
    decay = remaining - stable

    def factor(step: int) -> float:
        if step < num_warmup_steps:
            return float(step) / float(max(1, num_warmup_steps))
        if step < num_warmup_steps + stable:
            return 1.0
        if step < num_training_steps:
            progress = float(step - num_warmup_steps - stable) / float(max(1, decay))
            value = max(0.0, 0.5 * (1.0 + math.cos(math.pi * float(num_cycles) * 2.0 * progress)))
            return (1.0 - min_lr_ratio) * value + min_lr_ratio
        return min_lr_ratio

    return LambdaLR(optimizer, factor, last_epoch)


def build_lr_scheduler(optimizer, optim_config, role: str = "actor", rank: int = 0):
    """The scheduler the reference's workers build next to the optimizer (actor:
    fsdp_workers.py:425-450, critic: :1149-1170): warmup steps from lr_warmup_steps, or from
    lr_warmup_steps_ratio x total_training_steps when negative; "constant" or "cosine"
    (the actor's cosine takes min_lr_ratio / num_cycles, the critic's uses the defaults)."""
    total_steps = optim_config.get("total_training_steps", 0)
    num_warmup_steps = int(optim_config.get("lr_warmup_steps", -1))
    warmup_style = optim_config.get("warmup_style", "constant")
    if num_warmup_steps < 0:
        num_warmup_steps = int(optim_config.get("lr_warmup_steps_ratio", 0.0) * total_steps)
    if rank == 0:  # the reference prints this; stderr keeps a driver's JSON stdout clean
        import sys

        print(f"Total steps: {total_steps}, num_warmup_steps: {num_warmup_steps}", file=sys.stderr)
    if warmup_style == "constant":
        return get_constant_schedule_with_warmup(optimizer=optimizer, num_warmup_steps=num_warmup_steps)
    if warmup_style == "cosine":
        if role == "actor":
            return get_cosine_schedule_with_warmup(optimizer=optimizer, num_warmup_steps=num_warmup_steps,
                                                   num_training_steps=total_steps,
                                                   min_lr_ratio=optim_config.get("min_lr_ratio", 0.0),
                                                   num_cycles=optim_config.get("num_cycles", 0.5))
        return get_cosine_schedule_with_warmup(optimizer=optimizer, num_warmup_steps=num_warmup_steps,
                                               num_training_steps=total_steps)
    raise NotImplementedError(f"Warmup style {warmup_style} is not supported")
