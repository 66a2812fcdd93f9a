"""Collectives of the data-parallel path, in one place.

One process per GPU. Under RCCL (torch.distributed backend "nccl" on ROCm, over xGMI) device
tensors travel directly and RCCL's native AVG does the rank mean in the reduction (FSDP's fp32
mean, fsdp_workers.py:340-347); under gloo (CPU tests, or several ranks sharing one GPU in a
rehearsal) device tensors are staged through host memory and AVG is SUM then 1/W.

Every collective the step issues goes through these functions, and each one takes exactly one
of two branches on ``device_backend(group)``. The RCCL branch is therefore also what
``tests/_nccl_emulation.py`` drives on CPU at world size 8: it reports the backend as "nccl" and
maps AVG / reduce-scatter / all-gather-into-tensor onto gloo equivalents, so the bucket, ZeRO and
device-staging code that only RCCL reaches runs before the first multi-GPU launch. Call these as
``comm.<name>`` (module attribute), never ``from comm import``: the emulation patches
``comm_device``.
"""

from __future__ import annotations

import torch
import torch.distributed as dist


def initialized() -> bool:
    return dist.is_available() and dist.is_initialized()


def world(group=None) -> int:
    return dist.get_world_size(group) if initialized() else 1


def rank(group=None) -> int:
    return dist.get_rank(group) if initialized() else 0


def device_backend(group=None) -> bool:
    """True when the process group moves device tensors itself (RCCL)."""
    return initialized() and dist.get_backend(group) == "nccl"


def comm_device(group=None) -> torch.device:
    """Where small exchanged tensors (statistics, keys, checksums) must live for this group."""
    if device_backend(group):
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def _staged(t: torch.Tensor, group) -> bool:
    return t.is_cuda and not device_backend(group)


def all_reduce(t: torch.Tensor, op=dist.ReduceOp.SUM, group=None) -> torch.Tensor:
    """In-place all-reduce of ``t`` (any device); AVG is the mean over ranks. Returns ``t``."""
    if world(group) == 1:
        return t
    avg = op == dist.ReduceOp.AVG
    if avg and not t.is_floating_point():
        raise TypeError(f"all_reduce AVG needs a floating-point tensor, got {t.dtype}")
    if device_backend(group):
        dist.all_reduce(t, op=op, group=group)
        return t
    h = t.cpu() if t.is_cuda else t
    dist.all_reduce(h, op=dist.ReduceOp.SUM if avg else op, group=group)
    if avg:
        h.div_(world(group))
    if h is not t:
        t.copy_(h)
    return t


class _Done:
    """A finished collective (world size 1)."""

    def wait(self):
        return None


class _ScaleOnWait:
    """gloo has no AVG: the SUM's handle, scaled by 1/W when waited for."""

    def __init__(self, work, buf, scale):
        self.work, self.buf, self.scale = work, buf, scale

    def wait(self):
        self.work.wait()
        self.buf.mul_(self.scale)


class _HostStaged:
    """gloo on a device tensor: host copy, all-reduce, copy back (synchronous, at wait)."""

    def __init__(self, buf, group, avg):
        self.buf, self.group, self.avg = buf, group, avg

    def wait(self):
        all_reduce(self.buf, dist.ReduceOp.AVG if self.avg else dist.ReduceOp.SUM, self.group)


def all_reduce_mean_async(buf: torch.Tensor, group=None):
    """Start the mean over ranks of ``buf`` in place; returns a handle with ``wait()``."""
    w = world(group)
    if w == 1:
        return _Done()
    if device_backend(group):
        return dist.all_reduce(buf, op=dist.ReduceOp.AVG, group=group, async_op=True)
    if buf.is_cuda:
        return _HostStaged(buf, group, avg=True)
    return _ScaleOnWait(dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group, async_op=True), buf, 1.0 / w)


class _GlooReduceScatter:
    """gloo has no reduce-scatter: all-reduce the bucket (on the host) and keep this rank's shard."""

    def __init__(self, out, buf, group):
        self.out, self.buf, self.group = out, buf, group

    def wait(self):
        w, r = world(self.group), rank(self.group)
        host = self.buf.detach().cpu() if self.buf.is_cuda else self.buf.detach().clone()
        dist.all_reduce(host, op=dist.ReduceOp.SUM, group=self.group)
        n = self.out.numel()
        self.out.copy_(host[r * n : (r + 1) * n].to(self.out.device))
        self.out.mul_(1.0 / w)


def reduce_scatter_mean_async(out: torch.Tensor, buf: torch.Tensor, group=None):
    """out = mean over ranks of this rank's 1/W slice of buf (buf.numel() == W * out.numel())."""
    if world(group) == 1:
        out.copy_(buf)
        return _Done()
    if device_backend(group):
        return dist.reduce_scatter_tensor(out, buf, op=dist.ReduceOp.AVG, group=group, async_op=True)
    return _GlooReduceScatter(out, buf, group)


def all_gather_into(out: torch.Tensor, inp: torch.Tensor, group=None) -> None:
    """out (W * n elements) = the ranks' ``inp`` (n elements) in rank order."""
    w = world(group)
    if w == 1:
        out.copy_(inp.reshape(out.shape))
        return
    if device_backend(group):
        dist.all_gather_into_tensor(out, inp, group=group)
        return
    src = inp.cpu() if inp.is_cuda else inp
    parts = [torch.empty_like(src) for _ in range(w)]
    dist.all_gather(parts, src, group=group)
    out.copy_(torch.cat(parts).reshape(out.shape).to(out.device))


def all_gather(t: torch.Tensor, group=None) -> list[torch.Tensor]:
    """Equal-shape all-gather; the parts come back on ``t``'s device."""
    w = world(group)
    if w == 1:
        return [t]
    if _staged(t, group):
        parts = [torch.empty_like(t, device="cpu") for _ in range(w)]
        dist.all_gather(parts, t.cpu(), group=group)
        return [p.to(t.device) for p in parts]
    parts = [torch.empty_like(t) for _ in range(w)]
    dist.all_gather(parts, t.contiguous(), group=group)
    return parts


def broadcast(t: torch.Tensor, src: int = 0, group=None) -> None:
    """Broadcast from the group's rank ``src`` in place."""
    if world(group) == 1:
        return
    g_src = dist.get_global_rank(group, src) if group is not None else src
    if _staged(t, group):
        c = t.detach().cpu()
        dist.broadcast(c, src=g_src, group=group)
        t.copy_(c)
    else:
        dist.broadcast(t, src=g_src, group=group)


def barrier(group=None) -> None:
    if world(group) > 1:
        dist.barrier(group=group)
