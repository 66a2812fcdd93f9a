"""Data-parallel gradient synchronisation for the actor update, over RCCL (xGMI) or gloo.

Replaces the FSDP gradient reduce-scatter of the reference (fsdp_workers.py:370-405, fp32
reduce dtype :340-347) with plain DP: every rank keeps full fp32 parameters and gradients.

Design (MI355X-first):
  * gradients live in a few large flat fp32 buckets (``param.grad`` is a view into a bucket,
    so autograd accumulates straight into the communication buffer: no pack/unpack copies);
  * buckets are ordered as backward produces gradients (reverse parameter order), so the
    all-reduce of a full bucket is issued from a post-accumulate-grad hook while backward is
    still computing the earlier layers — communication overlaps compute;
  * only the LAST micro-batch of a mini-batch syncs (grad accumulation is local);
  * bucket size defaults to 256 MiB: xGMI rings are per-link bound, so few large messages;
  * the result is the mean over ranks (SUM then scale by 1/W), FSDP's reduction.
"""

from __future__ import annotations

import torch
import torch.distributed as dist


class _Bucket:
    __slots__ = ("buf", "params", "pending", "handle")

    def __init__(self, buf, params):
        self.buf = buf
        self.params = params
        self.pending = len(params)
        self.handle = None


class GradBucketReducer:
    def __init__(self, params, bucket_bytes: int = 256 << 20, process_group=None):
        self.group = process_group
        self.world = dist.get_world_size(process_group) if dist.is_available() and dist.is_initialized() else 1
        self.params = [p for p in params if p.requires_grad]
        self.sync_enabled = False
        self._hooks = []
        self.buckets: list[_Bucket] = []
        # reverse order ~ the order in which backward finishes each parameter's gradient
        ordered = list(reversed(self.params))
        cur, cur_bytes = [], 0
        groups = []
        for p in ordered:
            nb = p.numel() * 4
            if cur and (cur_bytes + nb > bucket_bytes or p.device != cur[0].device):
                groups.append(cur)
                cur, cur_bytes = [], 0
            cur.append(p)
            cur_bytes += nb
        if cur:
            groups.append(cur)
        self._bucket_of = {}
        for g in groups:
            n = sum(p.numel() for p in g)
            buf = torch.zeros(n, dtype=torch.float32, device=g[0].device)
            off = 0
            for p in g:
                p.grad = buf[off : off + p.numel()].view_as(p)
                off += p.numel()
            b = _Bucket(buf, g)
            self.buckets.append(b)
            for p in g:
                self._bucket_of[id(p)] = b
        if self.world > 1:
            for p in self.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))

    # ------------------------------------------------------------------ hooks
    def _on_grad(self, p):
        if not self.sync_enabled:
            return
        b = self._bucket_of[id(p)]
        b.pending -= 1
        if b.pending == 0:
            b.handle = dist.all_reduce(b.buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    # ------------------------------------------------------------------ API
    def zero_grad(self):
        for b in self.buckets:
            b.buf.zero_()
            for p in b.params:
                if p.grad is None or p.grad.data_ptr() < b.buf.data_ptr():
                    raise RuntimeError("a gradient view was replaced; use GradBucketReducer.zero_grad()")

    def begin_sync(self):
        """Call before the backward of the last micro-batch of a mini-batch."""
        self.sync_enabled = self.world > 1
        for b in self.buckets:
            b.pending = len(b.params)
            b.handle = None

    def finish_sync(self):
        """Wait for the bucket all-reduces and average; call after that backward."""
        if self.world <= 1:
            self.sync_enabled = False
            return
        for b in self.buckets:
            if b.handle is None:  # a parameter received no gradient in this backward
                b.handle = dist.all_reduce(b.buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        for b in self.buckets:
            b.handle.wait()
            b.buf.mul_(1.0 / self.world)
            b.handle = None
        self.sync_enabled = False

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks.clear()
