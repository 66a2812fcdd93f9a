"""Data-parallel advantage estimation: each rank computes advantages for its own shard.

The reference computes advantages on the driver over the whole batch (ray_trainer.py:214-291).
Sharded over W ranks this is exact when the only batch-global quantity is exchanged:

  * GRPO / RLOO: groups (prompts) are kept intact on one rank, so no exchange;
    ``check_groups_intact`` verifies it with one all_gather of the uid sets;
  * GAE / RF++-baseline whitening (torch_functional.py:206-223) is batch-global: each rank
    merges its rows' (count, sum, M2) into one fp64 triple on the device, the W triples are
    all-gathered (24 bytes per rank), and every rank merges them in rank order with the same
    kernel, so all ranks apply identical (mean, rstd) — bitwise equal to a single-process run
    over the rows in that order up to the merge tree.
"""

from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from ... import _lib as L
from ... import kernels as K


def _world(group) -> int:
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


def global_whiten_stats(local_merged: torch.Tensor, group=None) -> torch.Tensor:
    """local (n, sum, M2) fp64[3] on the device -> global fp32 stats {mean, rstd, n, flag}."""
    w = _world(group)
    dev = local_merged.device
    if w > 1:
        parts = [torch.empty_like(local_merged) for _ in range(w)]
        if dist.get_backend(group) == "gloo":  # gloo moves host tensors; keep the protocol identical
            cpu = [p.cpu() for p in parts]
            dist.all_gather(cpu, local_merged.cpu(), group=group)
            parts = [p.to(dev) for p in cpu]
        else:
            dist.all_gather(parts, local_merged, group=group)
        triples = torch.stack(parts).contiguous()
    else:
        triples = local_merged.view(1, 3).contiguous()
    stats = torch.empty(4, dtype=torch.float32, device=dev)
    merged = torch.empty(3, dtype=torch.float64, device=dev)
    L.call("va_whiten_finalize", K._p(triples), triples.shape[0], K._p(merged), K._p(stats), K._stream(stats))
    return stats


def masked_whiten_dp(values, mask, group=None, post_multiply_mask: bool = False):
    """masked_whiten over the union of all ranks' rows."""
    _, merged = K.whiten_stats(values, mask)
    stats = global_whiten_stats(merged, group)
    K._raise_whiten_flag(stats)
    return K.whiten_apply(values, mask, stats, post_multiply_mask=post_multiply_mask)


def compute_gae_advantage_return_dp(token_level_rewards, values, response_mask, gamma, lam, group=None):
    """GAE on this rank's rows; whitening statistics over all ranks (one 24-byte all-gather)."""
    _require = K._require_device
    _require(token_level_rewards, values, response_mask)
    r, v = K._f32(token_level_rewards), K._f32(values)
    B, R = r.shape
    m, mcode = K._mask(response_mask)
    adv = torch.empty_like(r)
    ret = torch.empty_like(r)
    part = torch.empty(B * 3 + 3, dtype=torch.float64, device=r.device)
    s = K._stream(r)
    with torch.no_grad():
        L.call("va_gae_scan", K._p(r), K._p(v), K._p(m), mcode, B, R, float(gamma), float(lam), K._p(adv), K._p(ret),
               K._p(part), s)
        local = part[B * 3:]
        stats4 = torch.empty(4, dtype=torch.float32, device=r.device)
        L.call("va_whiten_finalize", K._p(part), B, K._p(local), K._p(stats4), s)
        stats = global_whiten_stats(local, group)
        K._raise_whiten_flag(stats)
        L.call("va_whiten_apply", K._p(adv), K._p(stats), None, 0, B, R, 0, s)
    return adv, ret


def check_groups_intact(index, group=None) -> bool:
    """True when no uid appears on more than one rank (GRPO needs no exchange then)."""
    w = _world(group)
    if w == 1:
        return True
    mine = sorted(set(np.asarray(index).tolist()))
    allsets: list = [None] * w
    dist.all_gather_object(allsets, mine, group=group)
    seen: set = set()
    for s in allsets:
        if seen.intersection(s):
            return False
        seen.update(s)
    return True
