"""Run the RCCL-only branches of the data-parallel path on CPU (gloo) ranks.

``verl_amd.utils.comm`` takes its "nccl" branch whenever the process group reports that backend:
native AVG all-reduces, ``reduce_scatter_tensor`` (AVG) for the ZeRO buckets,
``all_gather_into_tensor`` for the bf16 weight shards, and small exchanges staged on
``comm_device()``. gloo provides none of AVG / reduce-scatter / all-gather-into-tensor, so without
help those lines only ever run on a real multi-GPU node. ``enable()`` makes a gloo world look like
RCCL to that code:

  * ``dist.get_backend`` reports "nccl";
  * ``dist.all_reduce(op=AVG)`` becomes SUM then 1/W (on ``wait()`` when asynchronous);
  * ``dist.reduce_scatter_tensor`` becomes an all-reduce of a copy, then this rank's slice;
  * ``dist.all_gather_into_tensor`` becomes ``all_gather`` + concatenation;
  * ``comm.comm_device`` returns the CPU (the staging device RCCL would need is a GPU).

Every emulated call is counted in ``CALLS`` so a test can assert that the branch ran.
Test infrastructure only; imported by tests, never by the product package.
"""

from __future__ import annotations

import collections

import torch
import torch.distributed as dist

CALLS: collections.Counter = collections.Counter()
_ORIG: dict = {}


class _AvgWork:
    def __init__(self, work, t, w):
        self.work, self.t, self.w = work, t, w

    def wait(self):
        self.work.wait()
        self.t.div_(self.w)
        return True


class _DoneWork:
    def wait(self):
        return True


def _all_reduce(tensor, op=dist.ReduceOp.SUM, group=None, async_op=False):
    if op == dist.ReduceOp.AVG:
        CALLS["all_reduce_avg"] += 1
        w = dist.get_world_size(group)
        work = _ORIG["all_reduce"](tensor, op=dist.ReduceOp.SUM, group=group, async_op=async_op)
        if async_op:
            return _AvgWork(work, tensor, w)
        tensor.div_(w)
        return None
    CALLS["all_reduce"] += 1
    return _ORIG["all_reduce"](tensor, op=op, group=group, async_op=async_op)


def _reduce_scatter_tensor(output, input, op=dist.ReduceOp.SUM, group=None, async_op=False):
    CALLS["reduce_scatter_tensor_avg" if op == dist.ReduceOp.AVG else "reduce_scatter_tensor"] += 1
    w, r = dist.get_world_size(group), dist.get_rank(group)
    assert input.numel() == w * output.numel(), (input.numel(), output.numel(), w)
    full = input.detach().clone()
    _ORIG["all_reduce"](full, op=dist.ReduceOp.SUM, group=group)
    n = output.numel()
    output.copy_(full.reshape(-1)[r * n : (r + 1) * n].reshape(output.shape))
    if op == dist.ReduceOp.AVG:
        output.div_(w)
    return _DoneWork() if async_op else None


def _all_gather_into_tensor(output_tensor, input_tensor, group=None, async_op=False):
    CALLS["all_gather_into_tensor"] += 1
    w = dist.get_world_size(group)
    assert output_tensor.numel() == w * input_tensor.numel()
    parts = [torch.empty_like(input_tensor) for _ in range(w)]
    dist.all_gather(parts, input_tensor.contiguous(), group=group)
    output_tensor.copy_(torch.cat([p.reshape(-1) for p in parts]).reshape(output_tensor.shape))
    return _DoneWork() if async_op else None


def _get_backend(group=None):
    return "nccl"


def enable():
    """Patch torch.distributed and verl_amd.utils.comm in THIS process (call after init)."""
    from verl_amd.utils import comm

    if _ORIG:
        return
    _ORIG.update(all_reduce=dist.all_reduce, reduce_scatter_tensor=dist.reduce_scatter_tensor,
                 all_gather_into_tensor=dist.all_gather_into_tensor, get_backend=dist.get_backend,
                 comm_device=comm.comm_device)
    dist.all_reduce = _all_reduce
    dist.reduce_scatter_tensor = _reduce_scatter_tensor
    dist.all_gather_into_tensor = _all_gather_into_tensor
    dist.get_backend = _get_backend
    comm.comm_device = lambda group=None: torch.device("cpu")


def disable():
    from verl_amd.utils import comm

    if not _ORIG:
        return
    dist.all_reduce = _ORIG["all_reduce"]
    dist.reduce_scatter_tensor = _ORIG["reduce_scatter_tensor"]
    dist.all_gather_into_tensor = _ORIG["all_gather_into_tensor"]
    dist.get_backend = _ORIG["get_backend"]
    comm.comm_device = _ORIG["comm_device"]
    _ORIG.clear()
