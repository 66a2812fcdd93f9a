"""Data-parallel gradient synchronisation for the actor update, over RCCL (xGMI) or gloo.

Replaces the FSDP gradient reduce-scatter of the reference (fsdp_workers.py:370-405, fp32
reduce dtype :340-347) with plain DP: every rank keeps full fp32 parameters and gradients.

Design (MI355X-first):
  * gradients live in a few large flat fp32 buckets (``param.grad`` is a view into a bucket,
    so autograd accumulates straight into the communication buffer: no pack/unpack copies);
  * buckets are ordered as backward produces gradients (reverse parameter order), so the
    all-reduce of a full bucket is issued from a post-accumulate-grad hook while backward is
    still computing the earlier layers — communication overlaps compute;
  * collectives are issued in ONE global order on every rank: bucket i is launched only after
    buckets 0..i-1 have been (a bucket that fills early waits for its predecessors), so ranks
    never issue RCCL calls in different orders;
  * only the LAST micro-batch of a mini-batch syncs (grad accumulation is local);
  * bucket size defaults to 256 MiB: xGMI rings are per-link bound, so few large messages;
  * the result is the mean over ranks (RCCL's native AVG; SUM then 1/W on gloo), FSDP's reduction;
  * at construction the parameters are broadcast from rank 0 (FSDP's sync_module_states), so
    replicas start identical whatever each rank's initialisation was.

``ShardedMixedPrecisionParams`` is the ZeRO-2-style variant: each
rank owns 1/W of every bucket's fp32 master weights and AdamW state, gradients are
reduce-scattered instead of all-reduced, and the updated bf16 shards are all-gathered back.
"""

from __future__ import annotations

import collections
import os
import weakref

import torch

from ..utils import comm


def _world_of(group) -> int:
    return comm.world(group)


def _rank_of(group) -> int:
    return comm.rank(group)


def _group_params(params, bucket_bytes: int, elem_bytes: int = 4):
    """Consecutive parameters (in backward order) packed into buckets of <= bucket_bytes."""
    groups, cur, cur_bytes = [], [], 0
    for p in params:
        nb = p.numel() * elem_bytes
        if cur and (cur_bytes + nb > bucket_bytes or p.device != cur[0].device):
            groups.append(cur)
            cur, cur_bytes = [], 0
        cur.append(p)
        cur_bytes += nb
    if cur:
        groups.append(cur)
    return groups



def _grad_hook(owner):
    """A post-accumulate-grad hook that calls ``owner._on_grad`` through a weak reference: a bound
    method stored on the parameters would keep the manager (and through it every parameter, master
    and gradient buffer) alive in a cycle the garbage collector cannot see through the autograd
    hooks, so a dropped worker would never free its device memory. The hook handles are removed
    when the owner is collected."""
    ref = weakref.WeakMethod(owner._on_grad)

    def hook(p):
        fn = ref()
        if fn is not None:
            fn(p)

    return hook


def _remove_hooks(handles):
    for h in handles:
        h.remove()

class _Bucket:
    __slots__ = ("buf", "params", "pending", "handle", "index", "ready")

    def __init__(self, buf, params, index):
        self.buf = buf
        self.params = params
        self.pending = len(params)
        self.handle = None
        self.index = index
        self.ready = False


class _OrderedBuckets:
    """Shared machinery: ordered asynchronous bucket collectives + optional timing."""

    group = None
    world = 1
    buckets: list

    def _init_order(self):
        self.sync_enabled = False
        self._next = 0
        self._timing = None
        # RCCL: native AVG in the reduction; gloo: SUM, then 1/W when waited for (utils/comm.py)
        self._use_avg = self.world > 1 and comm.device_backend(self.group)

    def _collective(self, b: _Bucket):
        """Start bucket b's all-reduce (mean over ranks)."""
        return comm.all_reduce_mean_async(b.buf, self.group)

    def _finish_bucket(self, b: _Bucket):
        b.handle.wait()

    def _mark_ready(self, b: _Bucket):
        """Bucket b is complete for this pass; launch every consecutive ready bucket in order."""
        b.ready = True
        while self._next < len(self.buckets) and self.buckets[self._next].ready:
            nb = self.buckets[self._next]
            nb.handle = self._collective(nb)
            self._next += 1

    def _reset_sync(self):
        self._next = 0
        for b in self.buckets:
            b.pending = len(b.params)
            b.handle = None
            b.ready = False

    def _finish_all(self):
        """Launch whatever has not been launched (in order), wait, average."""
        for b in self.buckets:
            b.ready = True
        if self.buckets:
            self._mark_ready(self.buckets[-1])
        ev0 = None
        if self._timing is not None:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev0.record()
        for b in self.buckets:
            self._finish_bucket(b)
            b.handle = None
        if ev0 is not None:
            ev1 = torch.cuda.Event(enable_timing=True)
            ev1.record()
            self._timing.append((ev0, ev1))
        self.sync_enabled = False

    # ------------------------------------------------------------------ measurement (bench.py)
    def start_timing(self):
        """Record, per optimizer step, the compute-stream time spent waiting for the gradient
        collectives after backward (the exposed, non-overlapped part)."""
        self._timing = []
        return self._timing

    def stop_timing(self) -> float:
        """Total exposed collective milliseconds since start_timing (synchronises)."""
        torch.cuda.synchronize()
        total = sum(a.elapsed_time(b) for a, b in (self._timing or []))
        self._timing = None
        return total

    def grad_bytes(self) -> int:
        return int(sum(b.buf.numel() * b.buf.element_size() for b in self.buckets))

    def time_isolated_sync(self, reps: int = 3) -> float:
        """Milliseconds of one step's gradient collectives run alone (no overlap), median of reps."""
        if self.world <= 1:
            return 0.0
        times = []
        for _ in range(reps + 1):
            scratch = [torch.zeros_like(b.buf) for b in self.buckets]
            comm.barrier(self.group)
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            hs = [self._raw_collective(s) for s in scratch]
            for h in hs:
                h.wait()
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1))
            del scratch
        return sorted(times[1:])[len(times[1:]) // 2]

    def _raw_collective(self, buf):
        return comm.all_reduce_mean_async(buf, self.group)


@torch.no_grad()
def _broadcast_from_rank0(tensors, group=None):
    """FSDP sync_module_states: every rank starts from rank 0's values."""
    for t in tensors:
        comm.broadcast(t, 0, group)


class GradBucketReducer(_OrderedBuckets):
    def __init__(self, params, bucket_bytes: int = 256 << 20, process_group=None, sync_params: bool = True):
        self.group = process_group
        self.world = _world_of(process_group)
        self.params = [p for p in params if p.requires_grad]
        self._hooks = []
        self.buckets: list[_Bucket] = []
        if sync_params:
            _broadcast_from_rank0([p.data for p in self.params], process_group)
        # reverse order ~ the order in which backward finishes each parameter's gradient
        groups = _group_params(list(reversed(self.params)), bucket_bytes)
        self._bucket_of = {}
        for i, g in enumerate(groups):
            n = sum(p.numel() for p in g)
            buf = torch.zeros(n, dtype=torch.float32, device=g[0].device)
            off = 0
            for p in g:
                p.grad = buf[off : off + p.numel()].view_as(p)
                off += p.numel()
            b = _Bucket(buf, g, i)
            self.buckets.append(b)
            for p in g:
                self._bucket_of[id(p)] = b
        self._init_order()
        if self.world > 1:
            for p in self.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(_grad_hook(self)))
            weakref.finalize(self, _remove_hooks, self._hooks)

    # ------------------------------------------------------------------ hooks
    def _on_grad(self, p):
        if not self.sync_enabled:
            return
        b = self._bucket_of[id(p)]
        b.pending -= 1
        if b.pending == 0:
            self._mark_ready(b)

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
        self._reset_sync()

    def finish_sync(self):
        """Wait for the bucket all-reduces and average; call after that backward."""
        if self.world <= 1:
            self.sync_enabled = False
            return
        self._finish_all()

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


class MixedPrecisionParams(_OrderedBuckets):
    """bf16 compute weights + fp32 master weights + fp32 gradient buckets.

    The MI355X equivalent of the reference's FSDP MixedPrecision(param_dtype=bf16,
    reduce_dtype=fp32, buffer_dtype=fp32) (fsdp_workers.py:337-347), without sharding:

      * the module's parameters are converted in place to bf16 (buffers such as RoPE's
        inv_freq stay fp32), so forward/backward run on bf16 weights with no per-op casts;
      * each parameter has an fp32 master copy living in a flat bucket; the optimizer (fused
        AdamW) and grad-norm clipping act on the masters;
      * after each parameter's bf16 gradient is produced, a post-accumulate-grad hook adds it
        into the fp32 bucket (accumulation over micro-batches in fp32) and frees it; on the last
        micro-batch the bucket's RCCL all-reduce is launched as soon as it and every bucket
        before it are full, overlapping communication with the rest of the backward;
      * after the optimizer step the masters are copied back to the bf16 weights (foreach copy).
    """

    def __init__(self, module: torch.nn.Module, bucket_bytes: int = 256 << 20, process_group=None,
                 compute_dtype=torch.bfloat16, sync_params: bool = True):
        self.group = process_group
        self.world = _world_of(process_group)
        self.compute_dtype = compute_dtype
        self.params = [p for p in module.parameters() if p.requires_grad]
        groups = _group_params(list(reversed(self.params)), bucket_bytes)
        self.buckets: list[_Bucket] = []
        self.master_bufs: list[torch.Tensor] = []
        self._master_of = {}
        self._gview = {}
        self._bucket_of = {}
        self._flat_of = {}  # id(master) -> (bucket index, element offset in its flat buffer)
        # FlatAdamW folds the clip's multiply and the next zero_grad into its step (see there)
        self.fold_clip = False
        self.clip_coef = None
        self._grads_zero = True
        for i, g in enumerate(groups):
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
                self._flat_of[id(master)] = (i, off)
                self._master_of[id(p)] = master
                self._gview[id(p)] = master.grad
                off += k
            self.master_bufs.append(mbuf)
            b = _Bucket(gbuf, g, i)
            self.buckets.append(b)
            for p in g:
                self._bucket_of[id(p)] = b
        if sync_params:
            _broadcast_from_rank0(self.master_bufs, process_group)
        # masters in module order (optimizer state order == parameter order)
        self.masters = [self._master_of[id(p)] for p in self.params]
        for p in self.params:
            p.data = self._master_of[id(p)].data.to(compute_dtype)
        self._ready: dict = {}
        self._init_order()
        self._hooks = [p.register_post_accumulate_grad_hook(_grad_hook(self)) for p in self.params]
        weakref.finalize(self, _remove_hooks, self._hooks)
        self.wgrad_stream = None
        self.side_stream_grads = 0  # gradients delivered on the side stream (tests / diagnostics)
        self._param_ids = {id(p) for p in self.params}
        self._side_ids = set()
        self._delivered = set()
        self._side_events = collections.deque()
        # how many side-stream weight-gradient launches may be outstanding before the compute stream
        # waits for the oldest (a GPU-side wait): bounds the activations / gradients the side stream
        # keeps alive when the compute stream's GEMMs starve it (unbounded lag -> +tens of GB)
        self.wgrad_max_lag = int(os.environ.get("VA_WGRAD_MAX_LAG", "4"))

    # ------------------------------------------------------------------ side-stream weight gradients
    def enable_wgrad_stream(self, params=None):
        """Run the weight gradients of ``params`` (the backbone projections, kernels._MergedLinear),
        every gradient accumulation into the fp32 buckets and the bucket collectives' launch on one
        side stream, so the backward's critical path (input gradients, attention, norms) overlaps
        them: a weight gradient whose GEMM leaves CUs idle (gate|up: 152 tiles of 256 x 256 for 256
        CUs) shares the chip with the next layer's input gradient. ``params`` must each receive
        their gradient from ONE use (a tied lm_head / embedding weight must not be listed). The
        compute stream waits for the side stream once per optimizer step (finish_sync)."""
        if not self.params or not self.params[0].is_cuda:
            return False
        if self.wgrad_stream is None:
            self.wgrad_stream = torch.cuda.Stream(device=self.params[0].device)
        allowed = self._param_ids if params is None else {id(p) for p in params}
        self._side_ids = allowed & self._param_ids
        return True

    def owns_exclusively(self, params) -> bool:
        """True when every parameter was listed in enable_wgrad_stream (one gradient source each)."""
        return self.wgrad_stream is not None and all(id(p) in self._side_ids for p in params)

    def deliver(self, params, grads):
        """Gradients produced on the side stream (the current stream of the caller)."""
        for p, g in zip(params, grads):
            if p.grad is not None:
                raise RuntimeError("side-stream weight gradient for a parameter that already has one")
            p.grad = g
            self.side_stream_grads += 1
            self._delivered.add(id(p))
            self._enqueue(p)

    def throttle(self, compute_stream, keep=()):
        """Called on the compute stream after each side-stream launch (kernels._MergedLinear).
        ``keep`` (the launch's compute-stream inputs) is released once the compute stream has been
        made to wait for the launch: from then on, stream-ordered reuse of their blocks by the
        compute stream is safe."""
        ev = torch.cuda.Event()
        ev.record(self.wgrad_stream)
        self._side_events.append((ev, keep))
        while len(self._side_events) > self.wgrad_max_lag:
            compute_stream.wait_event(self._side_events.popleft()[0])

    def _on_grad(self, p):
        if id(p) in self._delivered:
            # autograd still runs the parameter's AccumulateGrad (and this hook) for the None the
            # side-stream backward returned: the gradient was already handed over by deliver()
            self._delivered.discard(id(p))
            return
        self._enqueue(p)

    def _enqueue(self, p):
        b = self._bucket_of[id(p)]
        self._ready.setdefault(id(b), []).append(p)
        if len(self._ready[id(b)]) == len(b.params):
            self._flush_ordered(b)

    def _flush_ordered(self, b, complete: bool = True):
        side = self.wgrad_stream
        if side is None:
            self._flush(b, complete)
            return
        cur = torch.cuda.current_stream(side.device)
        if cur != side:
            side.wait_stream(cur)  # gradients made on the compute stream so far
        with torch.cuda.stream(side):
            self._flush(b, complete)

    def _flush(self, b, complete: bool = True):
        """Accumulate the bucket's ready bf16 gradients into its fp32 buffer (one multi-tensor
        launch) and, on a syncing micro-batch, mark it ready for its (ordered) collective."""
        ready = self._ready.pop(id(b), [])
        if ready:
            self._grads_zero = False
            if ready[0].is_cuda:
                from .. import kernels as K

                K.accumulate_grads([q.grad for q in ready], [self._gview[id(q)] for q in ready])
                if self.wgrad_stream is not None:
                    for q in ready:  # compute-stream gradients freed after the side stream reads them
                        q.grad.record_stream(self.wgrad_stream)
            else:
                for q in ready:
                    self._gview[id(q)].add_(q.grad)
            for q in ready:
                q.grad = None
        if complete and self.sync_enabled and not b.ready:
            self._mark_ready(b)

    def _join_wgrad_stream(self):
        if self.wgrad_stream is not None:
            torch.cuda.current_stream(self.wgrad_stream.device).wait_stream(self.wgrad_stream)
        self._side_events.clear()  # after the wait: the kept inputs may be reused in stream order

    def after_backward(self):
        """Flush buckets that did not complete (parameters without a gradient this pass)."""
        for b in self.buckets:
            if self._ready.get(id(b)):
                self._flush_ordered(b, complete=False)

    # same interface as GradBucketReducer
    def zero_grad(self):
        self._join_wgrad_stream()
        if not self._grads_zero:  # FlatAdamW's step already wrote the zeros
            for b in self.buckets:
                b.buf.zero_()
            self._grads_zero = True
        for p in self.params:
            p.grad = None
        self._ready = {}

    def flat_buckets(self) -> list:
        """(flat fp32 master buffer, flat fp32 gradient buffer) per bucket, in bucket order."""
        return [(m, b.buf) for m, b in zip(self.master_bufs, self.buckets, strict=True)]

    def flat_index(self, master) -> tuple:
        """(bucket index, element offset) of a master parameter inside flat_buckets()."""
        return self._flat_of[id(master)]

    def take_clip_coef(self):
        """The folded clip's coefficient (device scalar) once, or None."""
        c, self.clip_coef = self.clip_coef, None
        return c

    def grads_zeroed(self):
        """The optimizer step wrote zeros to every gradient bucket (FlatAdamW, zero_grad folded)."""
        self._grads_zero = True

    def begin_sync(self):
        self.sync_enabled = self.world > 1
        self._reset_sync()

    def finish_sync(self):
        self.after_backward()
        self._join_wgrad_stream()
        if self.world <= 1:
            self.sync_enabled = False
            return
        self._finish_all()

    def optimizer_params(self):
        return self.masters

    @torch.no_grad()
    def clip_grad_norm_(self, max_norm: float) -> torch.Tensor:
        """torch.nn.utils.clip_grad_norm_(masters, max_norm) (fsdp_utils.py:503-516 semantics: 2-norm
        of all gradients, coef = max_norm / (norm + 1e-6) clamped at 1, gradients scaled in place,
        the unclipped norm returned) over the flat fp32 buckets the masters' gradients tile without
        gaps: one reduction and one scale per bucket instead of one reduction per parameter (290
        per-parameter norms took ~5 ms per step on MI355X, the bucket norms ~0.5 ms)."""
        bufs = [b.buf for b in self.buckets]
        if not bufs:
            return torch.zeros(())
        total = torch.linalg.vector_norm(torch.stack(torch._foreach_norm(bufs)))
        coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
        if self.fold_clip:
            # FlatAdamW multiplies the gradients by coef as it reads them (the same fp32 product)
            self.clip_coef = coef
        else:
            torch._foreach_mul_(bufs, coef)
        return total

    @torch.no_grad()
    def after_step(self):
        """Refresh the bf16 compute weights from the fp32 masters."""
        torch._foreach_copy_([p.data for p in self.params], [m.data for m in self.masters])

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks.clear()


class FlatAdamW(torch.optim.Optimizer):
    """torch.optim.AdamW(fused=True) over a MixedPrecisionParams manager's fp32 masters, stepped as
    ONE streaming launch per flat bucket (va_adamw_flat, csrc/optim.hip) instead of torch's ~100
    multi-tensor launches over the ~290 per-parameter views (5.7 ms per step at ~2.4 TB/s,
    profiles/r06/d/kernel_stats_p8_summary.txt). The reference's _optimizer_step (dp_actor.py:272-288:
    clip_grad_norm_, a non-finite skip, optimizer.step(); AdamW from fsdp_workers.py:418-423):
      * torch's fused ADAMW arithmetic (its double-precision intermediates; tests/test_flat_adamw_gpu.py
        compares the masters and moments with torch.optim.AdamW(fused=True) bit for bit);
      * the gradient clip's in-place multiply is folded into the step (the manager keeps the
        coefficient, fold_clip), and so is the next zero_grad (the step writes zeros; the
        manager's zero_grad skips the buckets while nothing was accumulated since);
      * ``found_inf`` (a device flag, set by dp_actor.step_unless_nonfinite as for torch's fused
        AdamW) skips the update on the device: parameters, moments and the step count unchanged.
    The per-parameter state (exp_avg / exp_avg_sq / step) is exposed as views of the flat moments, in
    torch.optim.AdamW's layout. VERL_AMD_FLAT_ADAMW=0 keeps torch's AdamW (A/B runs)."""

    def __init__(self, manager, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 1e-2):
        params = manager.optimizer_params()
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay, amsgrad=False, maximize=False,
                        foreach=None, capturable=False, differentiable=False, fused=True)
        super().__init__(params, defaults)
        if len(self.param_groups) != 1:
            raise ValueError("FlatAdamW takes one parameter group (the manager's masters)")
        self.manager = manager
        self._flat = manager.flat_buckets()
        self._m = [torch.zeros_like(mf) for mf, _ in self._flat]
        self._v = [torch.zeros_like(mf) for mf, _ in self._flat]
        self._step = torch.zeros((), dtype=torch.float32, device=self._flat[0][0].device)
        self._bind_state(params)
        self.found_inf = None
        manager.fold_clip = True

    def _bind_state(self, params):
        for p in params:
            i, off = self.manager.flat_index(p)
            n = p.numel()
            self.state[p] = {"step": self._step, "exp_avg": self._m[i][off : off + n].view_as(p),
                             "exp_avg_sq": self._v[i][off : off + n].view_as(p)}

    def load_state_dict(self, state_dict):
        """torch.optim.Optimizer.load_state_dict, then the loaded moments and step copied into the flat
        buffers the kernel updates (the base class would leave the state as separate tensors)."""
        super().load_state_dict(state_dict)
        params = self.param_groups[0]["params"]
        step = None
        with torch.no_grad():
            for p in params:
                st = self.state.get(p, {})
                if "exp_avg" not in st:
                    continue
                i, off = self.manager.flat_index(p)
                n = p.numel()
                self._m[i][off : off + n].copy_(st["exp_avg"].reshape(-1))
                self._v[i][off : off + n].copy_(st["exp_avg_sq"].reshape(-1))
                step = st["step"]
            if step is not None:
                self._step.copy_(torch.as_tensor(step, dtype=torch.float32))
        self._bind_state(params)

    @torch.no_grad()
    def step(self, closure=None):
        from .. import _lib as L
        from .. import kernels as K

        loss = closure() if closure is not None else None
        g = self.param_groups[0]
        lr, (b1, b2), eps, wd = float(g["lr"]), g["betas"], float(g["eps"]), float(g["weight_decay"])
        fi = self.found_inf
        # torch's fused AdamW: step += 1, and -= found_inf after a skipped step
        self._step.add_(1.0) if fi is None else self._step.add_(1.0 - fi)
        coef = self.manager.take_clip_coef()
        st = K._stream(self._step)
        stream = torch.cuda.current_stream(self._step.device)
        for (mf, gf), m, v in zip(self._flat, self._m, self._v, strict=True):
            ev = K.TIMER.start(stream) if K.TIMER is not None else None
            L.call("va_adamw_flat", K._p(mf), K._p(gf), K._p(m), K._p(v), mf.numel(), lr, float(b1), float(b2), eps,
                   wd, K._p(self._step), K._p(coef) if coef is not None else None,
                   K._p(fi) if fi is not None else None, 1, st)
            if ev is not None:  # HBM-bound: p, g, m, v read, p, m, v, g (zeroed) written
                K.TIMER.stop("adamw_flat", 32 * mf.numel(), stream, ev)
        self.manager.grads_zeroed()
        return loss


class ShardedMixedPrecisionParams(_OrderedBuckets):
    """ZeRO-style data parallelism for the configs whose replicated optimizer state does not fit
    (Llama-3-8B actor + critic, Qwen2.5-7B DAPO; the reference shards with FSDP FULL_SHARD,
    fsdp_workers.py:94-99, 337-347, 371).

    Per rank, for P parameters over W ranks:
      * bf16 compute weights, full (2 P bytes): every parameter is a view into one flat bf16
        buffer per bucket, so the post-step all-gather writes straight into the weights;
      * fp32 gradient buckets, full (4 P bytes): bf16 micro-batch gradients accumulate into them
        (as MixedPrecisionParams) and, on the last micro-batch, each bucket is REDUCE-SCATTERED
        (RCCL AVG) in the fixed bucket order while backward continues;
      * fp32 master weights + AdamW moments for this rank's 1/W of every bucket (12 P / W bytes),
        as one flat parameter per bucket, so the fused AdamW runs over a few large tensors;
      * after the step each rank rounds its master shard to bf16 and the shards are
        all-gathered into the flat weight buffers.
    Gradient clipping uses the global norm (one fp32 all-reduce of the local sum of squares,
    fsdp2_clip_grad_norm_ fsdp_utils.py:503-516). AdamW is elementwise, so the updated weights
    equal those of replicated data parallelism."""

    def __init__(self, module: torch.nn.Module, bucket_bytes: int = 256 << 20, process_group=None,
                 compute_dtype=torch.bfloat16, sync_params: bool = True):
        self.group = process_group
        self.world = _world_of(process_group)
        self.rank = _rank_of(process_group)
        self.compute_dtype = compute_dtype
        self.params = [p for p in module.parameters() if p.requires_grad]
        groups = _group_params(list(reversed(self.params)), bucket_bytes)
        W = self.world
        self.buckets: list[_Bucket] = []
        self.flat_weights: list[torch.Tensor] = []
        self.shards: list[torch.nn.Parameter] = []
        self._gview = {}
        self._bucket_of = {}
        self._wslice = {}
        for i, g in enumerate(groups):
            n = sum(p.numel() for p in g)
            npad = -(-n // (W * 64)) * (W * 64)  # shards of whole 256-byte lines
            dev = g[0].device
            full = torch.zeros(npad, dtype=torch.float32, device=dev)
            off = 0
            for p in g:
                full[off : off + p.numel()].copy_(p.detach().reshape(-1).float())
                off += p.numel()
            if sync_params:
                _broadcast_from_rank0([full], process_group)
            gbuf = torch.zeros(npad, dtype=torch.float32, device=dev)
            wbuf = full.to(compute_dtype)
            off = 0
            for p in g:
                k = p.numel()
                self._gview[id(p)] = gbuf[off : off + k].view_as(p)
                p.data = wbuf[off : off + k].view_as(p)
                self._wslice[id(p)] = (i, off)
                off += k
            per = npad // W
            shard = torch.nn.Parameter(full[self.rank * per : (self.rank + 1) * per].clone(), requires_grad=True)
            shard.grad = torch.zeros(per, dtype=torch.float32, device=dev)
            del full
            self.flat_weights.append(wbuf)
            self.shards.append(shard)
            b = _Bucket(gbuf, g, i)
            self.buckets.append(b)
            for p in g:
                self._bucket_of[id(p)] = b
        self._ready: dict = {}
        self._init_order()
        self._hooks = [p.register_post_accumulate_grad_hook(_grad_hook(self)) for p in self.params]
        weakref.finalize(self, _remove_hooks, self._hooks)

    # ------------------------------------------------------------------ collectives
    def _collective(self, b: _Bucket):
        return comm.reduce_scatter_mean_async(self.shards[b.index].grad, b.buf, self.group)

    def _finish_bucket(self, b: _Bucket):
        b.handle.wait()

    def _raw_collective(self, buf):
        out = torch.empty(buf.numel() // self.world, dtype=buf.dtype, device=buf.device)
        return comm.reduce_scatter_mean_async(out, buf, self.group)

    # ------------------------------------------------------------------ hooks (as MixedPrecisionParams)
    def _on_grad(self, p):
        b = self._bucket_of[id(p)]
        self._ready.setdefault(id(b), []).append(p)
        if len(self._ready[id(b)]) == len(b.params):
            self._flush(b)

    def _flush(self, b, complete: bool = True):
        ready = self._ready.pop(id(b), [])
        if ready:
            self._grads_zero = False
            if ready[0].is_cuda:
                from .. import kernels as K

                K.accumulate_grads([q.grad for q in ready], [self._gview[id(q)] for q in ready])
            else:
                for q in ready:
                    self._gview[id(q)].add_(q.grad)
            for q in ready:
                q.grad = None
        if complete and self.sync_enabled and not b.ready:
            self._mark_ready(b)

    def after_backward(self):
        for b in self.buckets:
            if self._ready.get(id(b)):
                self._flush(b, complete=False)

    def zero_grad(self):
        for b in self.buckets:
            b.buf.zero_()
        for s in self.shards:
            s.grad.zero_()
        for p in self.params:
            p.grad = None
        self._ready = {}

    def begin_sync(self):
        self.sync_enabled = self.world > 1
        self._reset_sync()

    def finish_sync(self):
        self.after_backward()
        if self.world <= 1:  # one rank: the shard is the whole bucket
            for b in self.buckets:
                self.shards[b.index].grad.copy_(b.buf)
            self.sync_enabled = False
            return
        self._finish_all()

    def optimizer_params(self):
        return self.shards

    @torch.no_grad()
    def clip_grad_norm_(self, max_norm: float) -> torch.Tensor:
        """Global-norm clipping over the sharded gradients (torch.nn.utils.clip_grad_norm_
        semantics: coef = max_norm / (norm + 1e-6), clamped to 1; the norm is returned)."""
        grads = [s.grad for s in self.shards]
        local = torch.stack(torch._foreach_norm(grads)).square().sum()
        comm.all_reduce(local, group=self.group)
        norm = local.sqrt()
        coef = torch.clamp(max_norm / (norm + 1e-6), max=1.0)
        torch._foreach_mul_(grads, coef)
        return norm

    @torch.no_grad()
    def after_step(self):
        """Round the master shards to bf16 and all-gather them into the flat weight buffers; a
        parameter whose storage was re-pointed elsewhere since construction (the fused backbone
        merges q|k|v and gate|up into one buffer, qwen2_fused.py) gets its slice copied over."""
        for s, wbuf in zip(self.shards, self.flat_weights, strict=True):
            comm.all_gather_into(wbuf, s.detach().to(self.compute_dtype), self.group)
        dst, src = [], []
        for p in self.params:
            i, off = self._wslice[id(p)]
            wbuf = self.flat_weights[i]
            if p.data.data_ptr() != wbuf.data_ptr() + off * wbuf.element_size():
                dst.append(p.data)
                src.append(wbuf[off : off + p.numel()].view_as(p))
        if dst:
            torch._foreach_copy_(dst, src)

    def memory_bytes(self) -> dict:
        """Per-rank bytes of the parameter / gradient / optimizer state this manager holds."""
        w = sum(t.numel() * t.element_size() for t in self.flat_weights)
        g = sum(b.buf.numel() * 4 for b in self.buckets)
        m = sum(s.numel() * 4 for s in self.shards)
        return {"bf16_weights": w, "fp32_grads": g, "fp32_master_shard": m, "adamw_moments_shard": 2 * m}

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks.clear()
