"""End-of-run check that data-parallel replicas stayed identical.

The reference gets consistency by construction from FSDP (one sharded parameter set, gradients
reduced inside the wrapper, fsdp_workers.py:370-405). Here every rank owns its weights and the
update keeps them equal only if every rank applied the same averaged gradients and the same
optimizer step. ``replica_check`` proves it after a run: an order-independent integer checksum of
the bits of every compute weight (and of the fp32 masters when they are replicated) is reduced
with MAX and MIN over the ranks — equal means bit-identical replicas with overwhelming
probability — and the metrics that are global by definition (the clipped-gradient norm, the
learning rate) must be equal too.
"""

from __future__ import annotations

import torch
import torch.distributed as dist

from . import comm

_INT_VIEW = {1: torch.int8, 2: torch.int16, 4: torch.int32, 8: torch.int64}
_CHUNK = 1 << 24


def bits_checksum(tensors) -> torch.Tensor:
    """int64 [1]: sum over all elements of (raw bits, sign-extended) x (1 + position mod 8191),
    in wrapping int64 arithmetic, so the value does not depend on reduction order, and a single
    flipped bit or swapped pair of elements changes it."""
    acc = None
    for t in tensors:
        flat = t.detach().contiguous().reshape(-1)
        if flat.numel() == 0:
            continue
        bits = flat.view(_INT_VIEW[flat.element_size()])
        for s in range(0, bits.numel(), _CHUNK):
            v = bits[s : s + _CHUNK].to(torch.int64)
            w = torch.arange(s, s + v.numel(), device=v.device, dtype=torch.int64).remainder_(8191).add_(1)
            part = (v * w).sum().reshape(1)
            acc = part if acc is None else acc + part
    if acc is None:
        acc = torch.zeros(1, dtype=torch.int64)
    return acc


def replica_check(module: torch.nn.Module, manager=None, metrics: dict | None = None, metric_keys=(),
                  step_time_spread_s: float | None = None, group=None) -> dict:
    """Compare this rank's model and global metrics with every other rank's. ``manager``: the
    parameter manager (grad_sync.*); its fp32 masters are compared too unless they are sharded.
    Returns a dict with ``replicas_identical`` and the pieces; world size 1 is trivially identical."""
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    weights = list(module.parameters())
    sharded = manager is not None and hasattr(manager, "shards")
    masters = [] if manager is None or sharded else list(manager.optimizer_params())
    cs = torch.cat([bits_checksum(weights).cpu(), bits_checksum(masters).cpu()])
    keys = [k for k in metric_keys if metrics and k in metrics]
    vals = []
    for k in keys:
        v = metrics[k]
        vals.append(float(v[-1] if isinstance(v, (list, tuple)) else v))
    out = {
        "world": world,
        "weights_checksum": int(cs[0]),
        "masters_checked": bool(masters),
        "masters_sharded": sharded,
        "metrics_checked": keys,
        "step_time_spread_s": None if step_time_spread_s is None else round(step_time_spread_s, 4),
    }
    if world == 1:
        out.update(weights_equal=True, masters_equal=True, metrics_equal=True, replicas_identical=True)
        return out
    dev = comm.comm_device(group)
    hi, lo = cs.to(dev), cs.clone().to(dev)
    comm.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    comm.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    m = torch.tensor(vals, dtype=torch.float64)
    mh, ml = m.to(dev), m.clone().to(dev)
    if keys:
        comm.all_reduce(mh, op=dist.ReduceOp.MAX, group=group)
        comm.all_reduce(ml, op=dist.ReduceOp.MIN, group=group)
    hi, lo, mh, ml = hi.cpu(), lo.cpu(), mh.cpu(), ml.cpu()
    w_eq = bool(hi[0] == lo[0])
    m_eq = bool(hi[1] == lo[1])
    met_eq = bool(torch.equal(mh, ml)) if keys else True
    out.update(weights_equal=w_eq, masters_equal=m_eq, metrics_equal=met_eq,
               replicas_identical=w_eq and m_eq and met_eq,
               metrics_max_minus_min={k: float(a - b) for k, a, b in zip(keys, mh.tolist(), ml.tolist(), strict=True)})
    return out
