"""PyTorch-ROCm custom operators over the C-ABI of include/verl_amd.h.

Every hot-path kernel is registered as ``torch.ops.verl_amd.<name>`` with torch.library: a HIP
implementation (device_types="cuda": ROCm devices, no CPU kernel — a CPU tensor fails loudly in
the dispatcher), a fake (meta) implementation for tracing, and, for the differentiable ones,
an autograd formula that calls the matching backward op. The reference compiles
``entropy_from_logits`` with torch.compile by default (dp_actor.py:74-75); these registrations
let torch.compile trace the log-prob / loss wrappers without graph breaks.

Conventions shared by all ops:
  * inputs arrive in the layout the kernels read (the Python wrappers in kernels.py convert:
    fp32 contiguous for the [B, R] quantities, int64 labels, a mask of a supported dtype);
  * outputs and workspaces are allocated here from the torch caching allocator on the input's
    device; launches go to torch's current stream of that device; nothing synchronises;
  * scalar arguments are Python floats / ints; the C-ABI's ``float`` parameters round them to
    fp32 exactly as torch.clamp casts its scalar bounds (ctypes c_float conversion).

Op list (forward / backward pairs are wired by register_autograd):
  logprob_entropy_fwd, logprob_entropy_bwd, logprob_entropy_bwd_ (in place)
  ppo_loss_fwd, ppo_loss_bwd          (vanilla / gpg / clip_cov / kl_cov policy loss + KL + entropy)
  kl_penalty_fwd, kl_penalty_bwd
  masked_agg_fwd, masked_agg_bwd
  outcome_advantage (grpo_group_adv), row_scores, group_coef, broadcast_rows
  gae_scan, masked_row_partials, whiten_finalize, whiten_apply, gae_advantage_return
  apply_kl_penalty, discounted_returns
  value_loss_fwd, value_loss_bwd
"""

from __future__ import annotations

from typing import Optional

import torch
from torch import Tensor
from torch.library import custom_op

from . import _lib as L
from . import kernels as K

_NS = "verl_amd"
_F32 = torch.float32
_F64 = torch.float64


def _op(name, mutates_args=()):
    return custom_op(f"{_NS}::{name}", mutates_args=mutates_args, device_types="cuda")


def _check_f32(*ts):
    for t in ts:
        if t is not None and (t.dtype != _F32 or not t.is_contiguous()):
            raise TypeError(f"verl_amd op expects contiguous fp32 tensors, got {t.dtype}")


def _mcode(mask: Tensor) -> int:
    code = K._MASK_CODES.get(mask.dtype)
    if code is None or not mask.is_contiguous():
        raise TypeError(f"verl_amd op: unsupported / non-contiguous mask ({mask.dtype})")
    return code


def _rows(t: Tensor) -> tuple[int, int]:
    return K._as_2d(t)


# =============================================================================== log-prob + entropy
# backward_mode of logprob_entropy_fwd: where its backward writes dlogits
BWD_OUT_OF_PLACE = 0  # a fresh buffer (the stream runs ~3 % faster than in place)
BWD_IN_PLACE = 1  # over the logits (flash-attn inplace_backward, torch_functional.py:64-100)
BWD_AUTO = 2  # a fresh buffer when it can be allocated, else in place (the reference's path)


@_op("logprob_entropy_fwd")
def logprob_entropy_fwd(logits: Tensor, labels: Tensor, temperature: float,
                        backward_mode: int) -> tuple[Tensor, Tensor, Tensor]:
    """(logp, entropy, lse) fp32 [n] of logits [n, V] (row stride >= V, unit column stride);
    ``backward_mode`` (BWD_*) selects where the backward writes dlogits."""
    if logits.dim() != 2 or logits.stride(1) != 1:
        raise ValueError("logprob_entropy_fwd: logits must be [n, V] with unit column stride")
    if logits.dtype not in K._DTYPE_CODES:
        raise TypeError(f"unsupported logits dtype {logits.dtype}")
    n, V = logits.shape
    if labels.dtype != torch.int64 or labels.numel() != n or not labels.is_contiguous():
        raise ValueError("logprob_entropy_fwd: labels must be contiguous int64 [n]")
    logp = torch.empty(n, dtype=_F32, device=logits.device)
    ent = torch.empty(n, dtype=_F32, device=logits.device)
    lse = torch.empty(n, dtype=_F32, device=logits.device)
    if n == 0:
        return logp, ent, lse
    stream = torch.cuda.current_stream(logits.device)
    ev = K.TIMER.start(stream) if K.TIMER is not None else None
    L.call("va_logprob_entropy_fwd", K._p(logits), K._DTYPE_CODES[logits.dtype], n, V, logits.stride(0),
           K._p(labels), float(temperature), K._p(logp), K._p(ent), K._p(lse), K._vp(stream.cuda_stream))
    if ev is not None:  # algorithmic bytes: s*V logits + 8 label + 12 outputs per row
        K.TIMER.stop("logprob_entropy_fwd", n * (logits.element_size() * V + 20), stream, ev)
    return logp, ent, lse


@logprob_entropy_fwd.register_fake
def _(logits, labels, temperature, backward_mode):
    n = logits.shape[0]
    return (logits.new_empty(n, dtype=_F32), logits.new_empty(n, dtype=_F32), logits.new_empty(n, dtype=_F32))


def _lp_bwd_launch(g_logp, g_ent, logits, labels, lse, entropy, temperature, dx):
    n, V = logits.shape
    if n == 0:
        return
    _check_f32(g_logp, g_ent, lse, entropy)
    stream = torch.cuda.current_stream(logits.device)
    ev = K.TIMER.start(stream) if K.TIMER is not None else None
    L.call("va_logprob_entropy_bwd", K._p(g_logp), K._p(g_ent), K._p(logits), K._DTYPE_CODES[logits.dtype], n, V,
           logits.stride(0), K._p(labels), K._p(lse), K._p(entropy), float(temperature), K._p(dx), dx.stride(0),
           K._vp(stream.cuda_stream))
    if ev is not None:  # read + write logits, 28 B of row scalars
        K.TIMER.stop("logprob_entropy_bwd", n * (2 * logits.element_size() * V + 28), stream, ev)


@_op("logprob_entropy_bwd")
def logprob_entropy_bwd(g_logp: Optional[Tensor], g_ent: Optional[Tensor], logits: Tensor, labels: Tensor,
                        lse: Tensor, entropy: Tensor, temperature: float) -> Tensor:
    """dlogits (logits' dtype, dense [n, V]) = d(g_logp . logp + g_ent . H) / d logits."""
    dx = torch.empty(logits.shape, dtype=logits.dtype, device=logits.device)
    _lp_bwd_launch(g_logp, g_ent, logits, labels, lse, entropy, temperature, dx)
    return dx


@logprob_entropy_bwd.register_fake
def _(g_logp, g_ent, logits, labels, lse, entropy, temperature):
    return logits.new_empty(logits.shape)


@_op("logprob_entropy_bwd_", mutates_args=("logits",))
def logprob_entropy_bwd_(g_logp: Optional[Tensor], g_ent: Optional[Tensor], logits: Tensor, labels: Tensor,
                         lse: Tensor, entropy: Tensor, temperature: float) -> None:
    """In-place backward: dlogits overwrite the logits (flash-attn inplace_backward,
    torch_functional.py:64-100)."""
    _lp_bwd_launch(g_logp, g_ent, logits, labels, lse, entropy, temperature, logits)


@logprob_entropy_bwd_.register_fake
def _(g_logp, g_ent, logits, labels, lse, entropy, temperature):
    return None


def _lp_setup(ctx, inputs, output):
    logits, labels, temperature, mode = inputs
    _, ent, lse = output
    ctx.mark_non_differentiable(lse)
    ctx.save_for_backward(logits, labels, lse, ent)
    ctx.temperature = float(temperature)
    if int(mode) not in (BWD_OUT_OF_PLACE, BWD_IN_PLACE, BWD_AUTO):
        raise ValueError(f"logprob_entropy_fwd: backward_mode must be 0, 1 or 2, got {mode}")
    ctx.mode = int(mode)


# backward passes of BWD_AUTO that found no room for the dlogits buffer and wrote in place
AUTO_INPLACE_FALLBACKS = 0


def _lp_backward(ctx, g_logp, g_ent, g_lse):
    global AUTO_INPLACE_FALLBACKS
    logits, labels, lse, ent = ctx.saved_tensors
    g1 = None if g_logp is None else g_logp.float().contiguous()
    g2 = None if g_ent is None else g_ent.float().contiguous()
    mode = ctx.mode
    if mode == BWD_AUTO:
        # the caching allocator releases its cached blocks and retries before it raises, so an
        # OutOfMemoryError here means the buffer does not fit next to what is live: then dlogits
        # go over the logits as in the reference (the 196,608-token dynamic budget needs it)
        try:
            dx = torch.empty(logits.shape, dtype=logits.dtype, device=logits.device)
        except torch.OutOfMemoryError:
            dx = None
        if dx is not None:
            _lp_bwd_launch(g1, g2, logits, labels, lse, ent, ctx.temperature, dx)
            return dx, None, None, None
        AUTO_INPLACE_FALLBACKS += 1
        mode = BWD_IN_PLACE
    if mode == BWD_IN_PLACE:
        torch.ops.verl_amd.logprob_entropy_bwd_(g1, g2, logits, labels, lse, ent, ctx.temperature)
        return logits, None, None, None
    return torch.ops.verl_amd.logprob_entropy_bwd(g1, g2, logits, labels, lse, ent, ctx.temperature), None, None, None


logprob_entropy_fwd.register_autograd(_lp_backward, setup_context=_lp_setup)


# =============================================================================== policy loss
def _loss_ws(B: int, device, n_seg: int = 0) -> tuple[Tensor, Tensor]:
    # va_ppo_loss_workspace_bytes(B) / 8 doubles (= va_agg_workspace_bytes): the op returns the
    # leading B * 8 + 8 ([B, 8] row partials + 8 totals) + n_seg (the loss micro-batch segments'
    # token counts), every slot written by the forward; autograd saves it for the backward. The
    # tail is the forward's own per-workgroup scratch.
    buf = torch.empty(2 * B * 8 + 8, dtype=_F64, device=device)
    return buf, buf[: B * 8 + 8 + n_seg]


def _n_seg(B: int, seg_rows: int, seg_off: Optional[Tensor] = None) -> int:
    """Loss micro-batch segments of one launch: len(seg_off) - 1 (variable sizes), ceil(B / seg_rows)
    for 0 < seg_rows < B, else 0 (one aggregate)."""
    if seg_off is not None:
        return seg_off.numel() - 1
    return -(-B // seg_rows) if 0 < seg_rows < B else 0


def _check_seg_off(seg_off: Optional[Tensor], B: int):
    if seg_off is not None and (seg_off.dtype != torch.int32 or not seg_off.is_contiguous() or seg_off.dim() != 1
                                or not 2 <= seg_off.numel() <= B + 1):
        raise ValueError("seg_off must be a contiguous int32 [n_seg + 1] tensor of row offsets, 1 <= n_seg <= B")


def _loss_out_shape(B: int, seg_rows: int, seg_off: Optional[Tensor] = None, nout: int = L.VA_LOSS_NOUT) -> tuple:
    """[nout] for one aggregated batch; [S, nout] for S loss micro-batches (see _n_seg)."""
    S = _n_seg(B, seg_rows, seg_off)
    return (S, nout) if S else (nout,)


@_op("ppo_loss_fwd")
def ppo_loss_fwd(old_lp: Tensor, lp: Tensor, adv: Tensor, mask: Tensor, ref_lp: Optional[Tensor],
                 entropy: Optional[Tensor], sel: Optional[Tensor], clip_lo: float, clip_hi: float, clip_c: float,
                 agg_mode: int, kl_type: int, loss_mode: int, mode_coef: float,
                 seg_rows: int = 0, seg_off: Optional[Tensor] = None) -> tuple[Tensor, Tensor]:
    """(out fp32 = VA_LOSS_* slots, [8] or [S, 8] per loss micro-batch (seg_rows rows each, or the
    row ranges of seg_off); row-partials workspace fp64) of the fused policy loss."""
    _check_f32(old_lp, lp, adv, ref_lp, entropy)
    B, R = _rows(lp)
    if sel is not None and (sel.dtype != torch.uint8 or not sel.is_contiguous()):
        raise TypeError("ppo_loss_fwd: sel must be contiguous uint8")
    _check_seg_off(seg_off, B)
    out = torch.empty(_loss_out_shape(B, seg_rows, seg_off), dtype=_F32, device=lp.device)
    buf, ws = _loss_ws(B, lp.device, _n_seg(B, seg_rows, seg_off))
    L.call("va_ppo_loss_fwd", K._p(old_lp), K._p(lp), K._p(adv), K._p(mask), _mcode(mask), K._p(ref_lp),
           K._p(entropy), B, R, clip_lo, clip_hi, clip_c, agg_mode, kl_type, loss_mode, K._p(sel), mode_coef,
           seg_rows, K._p(seg_off), _n_seg(B, seg_rows, seg_off), K._p(out), K._p(buf), K._stream(lp))
    return out, ws


@ppo_loss_fwd.register_fake
def _(old_lp, lp, adv, mask, ref_lp, entropy, sel, clip_lo, clip_hi, clip_c, agg_mode, kl_type, loss_mode, mode_coef,
      seg_rows=0, seg_off=None):
    B = lp.numel() // lp.shape[-1] if lp.dim() > 1 else 1
    return (lp.new_empty(_loss_out_shape(B, seg_rows, seg_off), dtype=_F32),
            lp.new_empty(B * 8 + 8 + _n_seg(B, seg_rows, seg_off), dtype=_F64))


@_op("ppo_loss_bwd")
def ppo_loss_bwd(g_out: Tensor, old_lp: Tensor, lp: Tensor, adv: Tensor, mask: Tensor, ref_lp: Optional[Tensor],
                 sel: Optional[Tensor], ws: Tensor, clip_lo: float, clip_hi: float, clip_c: float, agg_mode: int,
                 kl_type: int, loss_mode: int, mode_coef: float, need_entropy: bool,
                 seg_rows: int = 0, seg_off: Optional[Tensor] = None) -> tuple[Tensor, Tensor]:
    """(d_lp [B, R] fp32, d_entropy [B, R] fp32 or [0] when not needed)."""
    _check_f32(g_out, old_lp, lp, adv, ref_lp)
    B, R = _rows(lp)
    _check_seg_off(seg_off, B)
    want = _loss_out_shape(B, seg_rows, seg_off)
    if g_out.shape != want:
        raise ValueError(f"ppo_loss_bwd: g_out shape {tuple(g_out.shape)} != {want}")
    d_lp = torch.empty(lp.shape, dtype=_F32, device=lp.device)
    d_ent = torch.empty(lp.shape if need_entropy else (0,), dtype=_F32, device=lp.device)
    L.call("va_ppo_loss_bwd", K._p(g_out), K._p(old_lp), K._p(lp), K._p(adv), K._p(mask), _mcode(mask), K._p(ref_lp),
           B, R, clip_lo, clip_hi, clip_c, agg_mode, kl_type, loss_mode, K._p(sel), mode_coef, seg_rows,
           K._p(seg_off), _n_seg(B, seg_rows, seg_off), K._p(ws), K._p(d_lp), K._p(d_ent) if need_entropy else None,
           K._stream(lp))
    return d_lp, d_ent


@ppo_loss_bwd.register_fake
def _(g_out, old_lp, lp, adv, mask, ref_lp, sel, ws, clip_lo, clip_hi, clip_c, agg_mode, kl_type, loss_mode,
      mode_coef, need_entropy, seg_rows=0, seg_off=None):
    return lp.new_empty(lp.shape), lp.new_empty(lp.shape if need_entropy else (0,))


def _loss_setup(ctx, inputs, output):
    old_lp, lp, adv, mask, ref_lp, entropy, sel, clip_lo, clip_hi, clip_c, agg, kl, mode, coef, seg_rows, seg_off = inputs
    _, ws = output
    ctx.mark_non_differentiable(ws)
    ctx.save_for_backward(old_lp, lp, adv, mask, ref_lp, sel, ws, seg_off)
    ctx.cfg = (clip_lo, clip_hi, clip_c, agg, kl, mode, coef, entropy is not None, seg_rows)


def _loss_backward(ctx, g_out, g_ws):
    old_lp, lp, adv, mask, ref_lp, sel, ws, seg_off = ctx.saved_tensors
    clip_lo, clip_hi, clip_c, agg, kl, mode, coef, has_ent, seg_rows = ctx.cfg
    need_ent = has_ent and ctx.needs_input_grad[5]
    d_lp, d_ent = torch.ops.verl_amd.ppo_loss_bwd(g_out.float().contiguous(), old_lp, lp, adv, mask, ref_lp, sel, ws,
                                                  clip_lo, clip_hi, clip_c, agg, kl, mode, coef, need_ent, seg_rows,
                                                  seg_off)
    return (None, d_lp if ctx.needs_input_grad[1] else None, None, None, None, d_ent if need_ent else None,
            None, None, None, None, None, None, None, None, None, None)


ppo_loss_fwd.register_autograd(_loss_backward, setup_context=_loss_setup)


# =============================================================================== KL penalty
@_op("kl_penalty_fwd")
def kl_penalty_fwd(lp: Tensor, ref: Tensor, kl_type: int) -> Tensor:
    _check_f32(lp, ref)
    out = torch.empty_like(lp)
    L.call("va_kl_penalty_fwd", K._p(lp), K._p(ref), lp.numel(), kl_type, K._p(out), K._stream(lp))
    return out


@kl_penalty_fwd.register_fake
def _(lp, ref, kl_type):
    return torch.empty_like(lp)


@_op("kl_penalty_bwd")
def kl_penalty_bwd(g: Tensor, lp: Tensor, ref: Tensor, kl_type: int) -> tuple[Tensor, Tensor]:
    _check_f32(g, lp, ref)
    d_lp = torch.empty_like(lp)
    d_ref = torch.empty_like(lp)
    L.call("va_kl_penalty_bwd", K._p(g), K._p(lp), K._p(ref), lp.numel(), kl_type, K._p(d_lp), K._p(d_ref),
           K._stream(lp))
    return d_lp, d_ref


@kl_penalty_bwd.register_fake
def _(g, lp, ref, kl_type):
    return torch.empty_like(lp), torch.empty_like(lp)


def _kl_setup(ctx, inputs, output):
    lp, ref, kl_type = inputs
    ctx.save_for_backward(lp, ref)
    ctx.kl_type = kl_type


def _kl_backward(ctx, g):
    lp, ref = ctx.saved_tensors
    d_lp, d_ref = torch.ops.verl_amd.kl_penalty_bwd(g.float().contiguous(), lp, ref, ctx.kl_type)
    return (d_lp if ctx.needs_input_grad[0] else None, d_ref if ctx.needs_input_grad[1] else None, None)


kl_penalty_fwd.register_autograd(_kl_backward, setup_context=_kl_setup)


# =============================================================================== masked aggregation
@_op("masked_agg_fwd")
def masked_agg_fwd(x: Tensor, mask: Tensor, mode: int) -> tuple[Tensor, Tensor]:
    """(out [1] or [B] for VA_REDUCE_ROW_MASKED_MEAN, workspace) of x [B, R] over the mask."""
    _check_f32(x)
    B, R = _rows(x)
    out = torch.empty(B if mode == L.VA_REDUCE_ROW_MASKED_MEAN else 1, dtype=_F32, device=x.device)
    buf, ws = _loss_ws(B, x.device)
    L.call("va_masked_agg_fwd", K._p(x), K._p(mask), _mcode(mask), B, R, mode, K._p(out), K._p(buf), K._stream(x))
    return out, ws


@masked_agg_fwd.register_fake
def _(x, mask, mode):
    B = x.numel() // x.shape[-1] if x.dim() > 1 else 1
    return x.new_empty(B if mode == L.VA_REDUCE_ROW_MASKED_MEAN else 1, dtype=_F32), x.new_empty(B * 8 + 8, dtype=_F64)


@_op("masked_agg_bwd")
def masked_agg_bwd(g: Tensor, mask: Tensor, mode: int, ws: Tensor) -> Tensor:
    _check_f32(g)
    B, R = _rows(mask)
    dx = torch.empty(mask.shape, dtype=_F32, device=mask.device)
    L.call("va_masked_agg_bwd", K._p(g), K._p(mask), _mcode(mask), B, R, mode, K._p(ws), K._p(dx), K._stream(mask))
    return dx


@masked_agg_bwd.register_fake
def _(g, mask, mode, ws):
    return mask.new_empty(mask.shape, dtype=_F32)


def _agg_setup(ctx, inputs, output):
    x, mask, mode = inputs
    ctx.mark_non_differentiable(output[1])
    ctx.save_for_backward(mask, output[1])
    ctx.mode = mode


def _agg_backward(ctx, g, g_ws):
    mask, ws = ctx.saved_tensors
    return torch.ops.verl_amd.masked_agg_bwd(g.float().contiguous(), mask, ctx.mode, ws), None, None


masked_agg_fwd.register_autograd(_agg_backward, setup_context=_agg_setup)


# =============================================================================== outcome advantages
@_op("outcome_advantage")
def outcome_advantage(rewards: Tensor, mask: Tensor, order: Tensor, offsets: Tensor, n_groups: int,
                      max_group_size: int, epsilon: float, estimator: int) -> Tensor:
    """grpo_group_adv: adv [B, R] = a(b) * mask for the GRPO-family estimator code (VA_ADV_*)."""
    _check_f32(rewards)
    B, R = rewards.shape
    adv = torch.empty_like(rewards)
    ws = torch.empty(3 * B, dtype=_F32, device=rewards.device)
    L.call("va_outcome_advantage", K._p(rewards), K._p(mask), _mcode(mask), B, R, K._p(order), K._p(offsets),
           n_groups, max_group_size, epsilon, estimator, K._p(adv), None, K._p(ws), K._stream(rewards))
    return adv


@outcome_advantage.register_fake
def _(rewards, mask, order, offsets, n_groups, max_group_size, epsilon, estimator):
    return torch.empty_like(rewards)


@_op("row_scores")
def row_scores(rewards: Tensor, mask: Optional[Tensor], with_lengths: bool) -> tuple[Tensor, Tensor]:
    """(scores [B], lengths [B] or [0]): unmasked reward row sums (+ response lengths)."""
    _check_f32(rewards)
    B, R = rewards.shape
    scores = torch.empty(B, dtype=_F32, device=rewards.device)
    lens = torch.empty(B if with_lengths else 0, dtype=_F32, device=rewards.device)
    mcode = _mcode(mask) if with_lengths else L.VA_MASK_F32
    L.call("va_row_scores", K._p(rewards), K._p(mask) if with_lengths else None, mcode, B, R, K._p(scores),
           K._p(lens) if with_lengths else None, K._stream(rewards))
    return scores, lens


@row_scores.register_fake
def _(rewards, mask, with_lengths):
    B = rewards.shape[0]
    return rewards.new_empty(B, dtype=_F32), rewards.new_empty(B if with_lengths else 0, dtype=_F32)


@_op("group_coef")
def group_coef(scores: Tensor, lengths: Optional[Tensor], order: Tensor, offsets: Tensor, n_groups: int,
               max_group_size: int, epsilon: float, estimator: int) -> Tensor:
    _check_f32(scores, lengths)
    coef = torch.empty_like(scores)
    L.call("va_group_coef", K._p(scores), K._p(lengths), K._p(order), K._p(offsets), n_groups, max_group_size,
           epsilon, estimator, K._p(coef), K._stream(scores))
    return coef


@group_coef.register_fake
def _(scores, lengths, order, offsets, n_groups, max_group_size, epsilon, estimator):
    return torch.empty_like(scores)


@_op("broadcast_rows")
def broadcast_rows(coef: Tensor, mask: Tensor) -> Tensor:
    _check_f32(coef)
    B, R = mask.shape
    if coef.numel() != B:
        raise ValueError(f"broadcast_rows: {coef.numel()} coefficients for {B} rows")
    adv = torch.empty(B, R, dtype=_F32, device=mask.device)
    L.call("va_broadcast_rows", K._p(coef), K._p(mask), _mcode(mask), B, R, K._p(adv), K._stream(adv))
    return adv


@broadcast_rows.register_fake
def _(coef, mask):
    return mask.new_empty(mask.shape, dtype=_F32)


# =============================================================================== GAE + whitening
def _gae_ws_doubles(B: int) -> int:
    return 6 * B + 8  # va_gae_workspace_bytes(B) / 8


@_op("gae_scan")
def gae_scan(rewards: Tensor, values: Tensor, mask: Tensor, gamma: float, lam: float) -> tuple[Tensor, Tensor, Tensor]:
    """(raw advantages, returns, workspace fp64 whose first va_gae_partial_count(B) triples are the
    partial (n, sum, M2) of the rows) — whitening not applied."""
    _check_f32(rewards, values)
    B, R = rewards.shape
    adv = torch.empty_like(rewards)
    ret = torch.empty_like(rewards)
    part = torch.zeros(_gae_ws_doubles(B), dtype=_F64, device=rewards.device)
    L.call("va_gae_scan", K._p(rewards), K._p(values), K._p(mask), _mcode(mask), B, R, gamma, lam, K._p(adv),
           K._p(ret), K._p(part), K._stream(rewards))
    return adv, ret, part


@gae_scan.register_fake
def _(rewards, values, mask, gamma, lam):
    B = rewards.shape[0]
    return torch.empty_like(rewards), torch.empty_like(rewards), rewards.new_empty(_gae_ws_doubles(B), dtype=_F64)


@_op("masked_row_partials")
def masked_row_partials(x: Tensor, mask: Tensor) -> Tensor:
    """fp64 [B*3 + 3]: per-row (n, sum, M2) of x over the mask (+ 3 slots for the merge)."""
    _check_f32(x)
    B, R = _rows(x)
    part = torch.zeros(B * 3 + 3, dtype=_F64, device=x.device)
    L.call("va_masked_row_partials", K._p(x), K._p(mask), _mcode(mask), B, R, K._p(part), K._stream(x))
    return part


@masked_row_partials.register_fake
def _(x, mask):
    B = x.numel() // x.shape[-1] if x.dim() > 1 else 1
    return x.new_empty(B * 3 + 3, dtype=_F64)


@_op("whiten_finalize")
def whiten_finalize(partials: Tensor, k: int) -> tuple[Tensor, Tensor]:
    """Merge the first k (n, sum, M2) triples in a fixed order: (merged fp64[3], stats fp32[4] =
    {mean, rsqrt(var + 1e-8), n, error_flag}). The partials are read from a private copy when the
    two-level merge (k > 1024) would overwrite them."""
    if k > 1024:
        partials = partials.clone()
    merged = torch.empty(3, dtype=_F64, device=partials.device)
    stats = torch.empty(4, dtype=_F32, device=partials.device)
    L.call("va_whiten_finalize", K._p(partials), k, K._p(merged), K._p(stats), K._stream(partials))
    return merged, stats


@whiten_finalize.register_fake
def _(partials, k):
    return partials.new_empty(3, dtype=_F64), partials.new_empty(4, dtype=_F32)


@_op("whiten_apply")
def whiten_apply(x: Tensor, stats: Tensor, mask: Optional[Tensor], post_multiply_mask: bool) -> Tensor:
    """(x - mean) * rstd [* mask] into a new tensor."""
    _check_f32(x)
    y = x.clone()
    B, R = _rows(y)
    mcode = _mcode(mask) if post_multiply_mask else 0
    L.call("va_whiten_apply", K._p(y), K._p(stats), K._p(mask) if post_multiply_mask else None, mcode, B, R,
           1 if post_multiply_mask else 0, K._stream(y))
    return y


@whiten_apply.register_fake
def _(x, stats, mask, post_multiply_mask):
    return torch.empty_like(x)


@_op("gae_advantage_return")
def gae_advantage_return(rewards: Tensor, values: Tensor, mask: Tensor, gamma: float,
                         lam: float) -> tuple[Tensor, Tensor, Tensor]:
    """(whitened advantages, returns, stats fp32[4]) — compute_gae_advantage_return."""
    _check_f32(rewards, values)
    B, R = rewards.shape
    adv = torch.empty_like(rewards)
    ret = torch.empty_like(rewards)
    stats = torch.empty(4, dtype=_F32, device=rewards.device)
    ws = torch.empty(_gae_ws_doubles(B), dtype=_F64, device=rewards.device)
    L.call("va_gae_advantage_return", K._p(rewards), K._p(values), K._p(mask), _mcode(mask), B, R, gamma, lam,
           K._p(adv), K._p(ret), K._p(stats), K._p(ws), K._stream(rewards))
    return adv, ret, stats


@gae_advantage_return.register_fake
def _(rewards, values, mask, gamma, lam):
    return torch.empty_like(rewards), torch.empty_like(rewards), rewards.new_empty(4, dtype=_F32)


# =============================================================================== in-reward KL, returns
@_op("apply_kl_penalty")
def apply_kl_penalty(scores: Tensor, old_lp: Tensor, ref_lp: Tensor, mask: Tensor, kl_type: int,
                     beta: float) -> tuple[Tensor, Tensor]:
    _check_f32(scores, old_lp, ref_lp)
    B, R = scores.shape
    rewards = torch.empty_like(scores)
    row_kl = torch.empty(B, dtype=_F32, device=scores.device)
    L.call("va_apply_kl_penalty", K._p(scores), K._p(old_lp), K._p(ref_lp), K._p(mask), _mcode(mask), B, R, kl_type,
           beta, K._p(rewards), K._p(row_kl), K._stream(scores))
    return rewards, row_kl


@apply_kl_penalty.register_fake
def _(scores, old_lp, ref_lp, mask, kl_type, beta):
    return torch.empty_like(scores), scores.new_empty(scores.shape[0], dtype=_F32)


@_op("discounted_returns")
def discounted_returns(rewards: Tensor, mask: Tensor, gamma: float, mode: int,
                       baselines: Optional[Tensor]) -> tuple[Tensor, Tensor]:
    """(returns, adv) — adv is [0] for REINFORCE++ (mode VA_RET_RFPP)."""
    _check_f32(rewards, baselines)
    B, R = rewards.shape
    ret = torch.empty_like(rewards)
    remax = mode == L.VA_RET_REMAX
    adv = torch.empty(rewards.shape if remax else (0,), dtype=_F32, device=rewards.device)
    L.call("va_discounted_returns", K._p(rewards), K._p(mask), _mcode(mask), B, R, gamma, mode, K._p(baselines),
           K._p(ret), K._p(adv) if remax else None, K._stream(rewards))
    return ret, adv


@discounted_returns.register_fake
def _(rewards, mask, gamma, mode, baselines):
    return torch.empty_like(rewards), rewards.new_empty(rewards.shape if mode == L.VA_RET_REMAX else (0,))


# =============================================================================== value loss (critic)
@_op("value_loss_fwd")
def value_loss_fwd(vpreds: Tensor, values: Tensor, returns: Tensor, mask: Tensor, cliprange_value: float,
                   agg_mode: int, seg_rows: int = 0, seg_off: Optional[Tensor] = None) -> tuple[Tensor, Tensor]:
    """(out fp32 = VA_VLOSS_* slots, [4] or [S, 4] per loss micro-batch (as ppo_loss_fwd); workspace)."""
    _check_f32(vpreds, values, returns)
    B, R = _rows(vpreds)
    _check_seg_off(seg_off, B)
    out = torch.empty(_loss_out_shape(B, seg_rows, seg_off, L.VA_VLOSS_NOUT), dtype=_F32, device=vpreds.device)
    buf, ws = _loss_ws(B, vpreds.device, _n_seg(B, seg_rows, seg_off))
    L.call("va_value_loss_fwd", K._p(vpreds), K._p(values), K._p(returns), K._p(mask), _mcode(mask), B, R,
           cliprange_value, agg_mode, seg_rows, K._p(seg_off), _n_seg(B, seg_rows, seg_off), K._p(out), K._p(buf),
           K._stream(vpreds))
    return out, ws


@value_loss_fwd.register_fake
def _(vpreds, values, returns, mask, cliprange_value, agg_mode, seg_rows=0, seg_off=None):
    B = vpreds.numel() // vpreds.shape[-1] if vpreds.dim() > 1 else 1
    return (vpreds.new_empty(_loss_out_shape(B, seg_rows, seg_off, L.VA_VLOSS_NOUT), dtype=_F32),
            vpreds.new_empty(B * 8 + 8 + _n_seg(B, seg_rows, seg_off), dtype=_F64))


@_op("value_loss_bwd")
def value_loss_bwd(g_out: Tensor, vpreds: Tensor, values: Tensor, returns: Tensor, mask: Tensor, ws: Tensor,
                   cliprange_value: float, agg_mode: int, seg_rows: int = 0,
                   seg_off: Optional[Tensor] = None) -> Tensor:
    _check_f32(g_out, vpreds, values, returns)
    B, R = _rows(vpreds)
    _check_seg_off(seg_off, B)
    want = _loss_out_shape(B, seg_rows, seg_off, L.VA_VLOSS_NOUT)
    if g_out.shape != want:
        raise ValueError(f"value_loss_bwd: g_out shape {tuple(g_out.shape)} != {want}")
    d = torch.empty_like(vpreds)
    L.call("va_value_loss_bwd", K._p(g_out), K._p(vpreds), K._p(values), K._p(returns), K._p(mask), _mcode(mask), B,
           R, cliprange_value, agg_mode, seg_rows, K._p(seg_off), _n_seg(B, seg_rows, seg_off), K._p(ws), K._p(d),
           K._stream(vpreds))
    return d


@value_loss_bwd.register_fake
def _(g_out, vpreds, values, returns, mask, ws, cliprange_value, agg_mode, seg_rows=0, seg_off=None):
    return torch.empty_like(vpreds)


def _vloss_setup(ctx, inputs, output):
    vpreds, values, returns, mask, c, agg, seg_rows, seg_off = inputs
    ctx.mark_non_differentiable(output[1])
    ctx.save_for_backward(vpreds, values, returns, mask, output[1], seg_off)
    ctx.cfg = (c, agg, seg_rows)


def _vloss_backward(ctx, g_out, g_ws):
    vpreds, values, returns, mask, ws, seg_off = ctx.saved_tensors
    c, agg, seg_rows = ctx.cfg
    d = torch.ops.verl_amd.value_loss_bwd(g_out.float().contiguous(), vpreds, values, returns, mask, ws, c, agg,
                                          seg_rows, seg_off)
    return d, None, None, None, None, None, None, None


value_loss_fwd.register_autograd(_vloss_backward, setup_context=_vloss_setup)


OPS = [
    "logprob_entropy_fwd", "logprob_entropy_bwd", "logprob_entropy_bwd_", "ppo_loss_fwd", "ppo_loss_bwd",
    "kl_penalty_fwd", "kl_penalty_bwd", "masked_agg_fwd", "masked_agg_bwd", "outcome_advantage", "row_scores",
    "group_coef", "broadcast_rows", "gae_scan", "masked_row_partials", "whiten_finalize", "whiten_apply",
    "gae_advantage_return", "apply_kl_penalty", "discounted_returns", "value_loss_fwd", "value_loss_bwd",
]
