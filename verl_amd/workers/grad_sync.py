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

    def optimizer_params(self):
        return self.params

    def after_backward(self):
        pass

    def after_step(self):
        pass

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks.clear()


class MixedPrecisionParams:
    """bf16 compute weights + fp32 master weights + fp32 gradient buckets.

    The MI355X equivalent of the reference's FSDP MixedPrecision(param_dtype=bf16,
    reduce_dtype=fp32, buffer_dtype=fp32) (fsdp_workers.py:337-347), without sharding:

      * the module's parameters are converted in place to bf16 (buffers such as RoPE's
        inv_freq stay fp32), so forward/backward run on bf16 weights with no per-op casts;
      * each parameter has an fp32 master copy living in a flat bucket; the optimizer (fused
        AdamW) and grad-norm clipping act on the masters;
      * after each parameter's bf16 gradient is produced, a post-accumulate-grad hook adds it
        into the fp32 bucket (accumulation over micro-batches in fp32) and frees it; on the last
        micro-batch the hook launches the bucket's RCCL all-reduce as soon as the bucket is full,
        overlapping communication with the rest of the backward;
      * after the optimizer step the masters are copied back to the bf16 weights (foreach copy).
    """

    def __init__(self, module: torch.nn.Module, bucket_bytes: int = 256 << 20, process_group=None,
                 compute_dtype=torch.bfloat16):
        self.group = process_group
        self.world = dist.get_world_size(process_group) if dist.is_available() and dist.is_initialized() else 1
        self.compute_dtype = compute_dtype
        self.params = [p for p in module.parameters() if p.requires_grad]
        self.sync_enabled = False
        ordered = list(reversed(self.params))
        groups, cur, cur_bytes = [], [], 0
        for p in ordered:
            nb = p.numel() * 4
            if cur and cur_bytes + nb > bucket_bytes:
                groups.append(cur)
                cur, cur_bytes = [], 0
            cur.append(p)
            cur_bytes += nb
        if cur:
            groups.append(cur)
        self.buckets: list[_Bucket] = []
        self.masters: list[torch.nn.Parameter] = []
        self._master_of = {}
        self._gview = {}
        self._bucket_of = {}
        for g in groups:
            n = sum(p.numel() for p in g)
            dev = g[0].device
            mbuf = torch.empty(n, dtype=torch.float32, device=dev)
            gbuf = torch.zeros(n, dtype=torch.float32, device=dev)
            off = 0
            for p in g:
                k = p.numel()
                mv = mbuf[off : off + k].view_as(p)
                mv.copy_(p.detach().float())
                master = torch.nn.Parameter(mv, requires_grad=True)
                master.grad = gbuf[off : off + k].view_as(p)
                self._master_of[id(p)] = master
                self._gview[id(p)] = master.grad
                off += k
            b = _Bucket(gbuf, g)
            self.buckets.append(b)
            for p in g:
                self._bucket_of[id(p)] = b
        # masters in module order (optimizer state order == parameter order)
        self.masters = [self._master_of[id(p)] for p in self.params]
        for p in self.params:
            p.data = p.data.to(compute_dtype)
        self._ready: dict = {}
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self.params]

    def _on_grad(self, p):
        b = self._bucket_of[id(p)]
        self._ready.setdefault(id(b), []).append(p)
        if len(self._ready[id(b)]) == len(b.params):
            self._flush(b)

    def _flush(self, b):
        """Accumulate the bucket's ready bf16 gradients into its fp32 buffer (one multi-tensor
        launch) and, on a syncing micro-batch, start the bucket's all-reduce."""
        ready = self._ready.pop(id(b), [])
        if ready:
            if ready[0].is_cuda:
                from .. import kernels as K

                K.accumulate_grads([q.grad for q in ready], [self._gview[id(q)] for q in ready])
            else:
                for q in ready:
                    self._gview[id(q)].add_(q.grad)
            for q in ready:
                q.grad = None
        if self.sync_enabled and b.handle is None and not self._ready.get(id(b)):
            b.handle = dist.all_reduce(b.buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def after_backward(self):
        """Flush buckets that did not complete (parameters without a gradient this pass)."""
        for b in self.buckets:
            if self._ready.get(id(b)):
                self._flush(b)

    # same interface as GradBucketReducer
    def zero_grad(self):
        for b in self.buckets:
            b.buf.zero_()
        for p in self.params:
            p.grad = None
        self._ready = {}

    def begin_sync(self):
        self.sync_enabled = self.world > 1
        for b in self.buckets:
            b.pending = len(b.params)
            b.handle = None

    def finish_sync(self):
        self.after_backward()
        if self.world <= 1:
            self.sync_enabled = False
            return
        for b in self.buckets:
            if b.handle is None:
                b.handle = dist.all_reduce(b.buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        for b in self.buckets:
            b.handle.wait()
            b.buf.mul_(1.0 / self.world)
            b.handle = None
        self.sync_enabled = False

    def optimizer_params(self):
        return self.masters

    @torch.no_grad()
    def after_step(self):
        """Refresh the bf16 compute weights from the fp32 masters."""
        torch._foreach_copy_([p.data for p in self.params], [m.data for m in self.masters])

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks.clear()
