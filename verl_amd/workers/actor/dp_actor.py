"""DataParallelPPOActor — mirror of verl/workers/actor/dp_actor.py:51-486 on MI355X.

Same constructor, config keys, micro/mini-batch loops, loss scaling and metric keys as the
reference. What changes is how the hot path maps onto the GPU:

  * padding removal is computed once per call on the host from the attention mask (one D2H
    copy), so the micro-batch loop has no host syncs;
  * the backbone runs on packed tokens with PyTorch-ROCm flash varlen attention
    (attention.py) and only the hidden states that predict response tokens go through the
    lm_head (the reference materialises logits for prompt tokens too and slices afterwards,
    dp_actor.py:219-237), with the reference's labels, so the returned log-probs and entropies
    equal its tensors at every position (masked ones included);
  * temperature, log-softmax, label gather and entropy are ONE fused gfx950 kernel pass over
    the logits (va_logprob_entropy_fwd); its backward writes dlogits in place (the reference's
    inplace_backward) or, with logprob_inplace_backward=False (the bench), into a fresh buffer;
  * Qwen2-VL (BASELINE config 4): mrope position ids [B, 3, S] pack to [3, T] and the fused
    backbone selects the rotary sections (qwen2_fused.rotary); multi_modal_inputs go through the
    model's own vision tower (HF; outside SURVEY §8) onto the placeholder tokens;
  * the clipped policy loss, KL loss, entropy aggregation and metrics are one fused kernel
    (va_ppo_loss_fwd/bwd); metrics stay on device and are read once per update;
  * gradients are averaged across DP ranks by a bucketed RCCL all-reduce overlapped with the
    last micro-batch's backward (grad_sync.py), then clipped and stepped (AdamW).
"""

from __future__ import annotations

import logging
import os
from collections.abc import MutableMapping
from dataclasses import dataclass

import numpy as np
import torch
from torch import nn

from ... import _lib as L
from ... import kernels as K
from ...protocol import DataProto
from ...trainer.ppo import core_algos
from ...trainer.ppo.core_algos import agg_loss, get_policy_loss_fn, kl_penalty
from ...utils import torch_functional as verl_F
from ...utils.seqlen_balancing import prepare_dynamic_batch, restore_dynamic_batch
from . import attention
from .base import BasePPOActor

__all__ = ["DataParallelPPOActor"]

logger = logging.getLogger(__file__)
logger.setLevel(os.getenv("VERL_LOGGING_LEVEL", "WARN"))

_NO_MASK = {"full_attention": None, "sliding_attention": None}


def packed_mask_arg(backbone):
    """attention_mask argument for an HF backbone run on packed tokens with the registered varlen
    attention: Qwen2 takes a per-layer-type mask mapping (None everywhere skips mask creation),
    other decoders (Llama) take None, which the registered no-op mask function keeps None."""
    return _NO_MASK if getattr(backbone.config, "model_type", "") == "qwen2" else None


def append_to_dict(data: dict, new_data: dict):
    for k, v in new_data.items():
        data.setdefault(k, []).append(v)


@dataclass
class _Packing:
    """Host-computed padding removal of one micro-batch (flash_attn.bert_padding.unpad_input)."""

    token_idx: torch.Tensor  # [nnz] flat indices of real tokens in [B*S]
    cu_seqlens: torch.Tensor  # [B+1] int32
    max_seqlen: int
    sel_hidden: torch.Tensor  # [n_sel] rows of the packed hidden states whose log-prob is kept
    sel_out: torch.Tensor  # [n_sel] flat index into [B*R]
    label_idx: torch.Tensor  # [n_sel] flat index into input_ids [B*S]: each selected row's label
    attn_blocks: torch.Tensor = None  # [n, 2] int32 (sequence, first query row) for va_flash_attn_fwd
    attn_kblocks: torch.Tensor = None  # [n, 2] int32 (sequence, first key) for va_flash_attn_bwd
    pad: int = 0  # dummy tokens appended as one extra sequence (pad_multiple)
    pad_pos: torch.Tensor = None  # [pad] int64 position ids of the dummy sequence

    def gather(self, input_ids: torch.Tensor, position_ids: torch.Tensor):
        """Packed (ids [T], pos [T]) of the real tokens, followed by the dummy sequence. Qwen2-VL's
        mrope position ids [B, 3, S] pack to [3, T] (dp_actor.py:106-121: (bsz, 3, seqlen) ->
        (3, bsz, seqlen) -> (3, total_nnz)); the dummy sequence gets 0..pad-1 on all three rows."""
        ids = input_ids.reshape(-1).index_select(0, self.token_idx)
        if position_ids.dim() == 3:
            c = position_ids.shape[1]
            pos = position_ids.transpose(0, 1).reshape(c, -1).index_select(1, self.token_idx)
        else:
            pos = position_ids.reshape(-1).index_select(0, self.token_idx)
        if self.pad:
            ids = torch.cat([ids, ids.new_zeros(self.pad)])
            pos = torch.cat([pos, self.pad_pos.expand(*pos.shape[:-1], self.pad)], dim=-1)
        return ids, pos


def _plan_packing(attn_mask_cpu: np.ndarray, R: int, device, pad_multiple: int = 0, groups=None) -> _Packing:
    """Padding removal of one micro-batch. With ``pad_multiple`` > 0 the packed length is rounded
    up to a multiple of it by one extra dummy sequence (token 0, positions 0..pad-1): the model
    GEMMs then see a few fixed token counts, so a tuned GEMM table (utils/gemm_tuning.py) applies.
    The dummy rows are never selected for the loss, so their gradients are exactly zero and they
    attend only to themselves: the real tokens' results and every weight gradient are unchanged.

    Selected rows and labels are the reference's (dp_actor.py:131-137, 219-237): position
    p = S - R - 1 + t gets log p(input_ids[p + 1]) when p is a real token, and 0 (pad_input) when it
    is padding. For the last real token of a row whose response is shorter than R, the label is the
    reference's rolled packed stream (torch.roll(input_ids_rmpad, -1)): the first real token of the
    next row of the reference's micro-batch, or of its first row for its last row. ``groups``: the
    row offsets of the reference's micro-batches inside this one ([0, B] when they coincide), e.g.
    the 8-row loss micro-batches of a 128-row update pass."""
    B, S = attn_mask_cpu.shape
    flat = attn_mask_cpu.reshape(-1).astype(bool)
    token_idx = np.flatnonzero(flat)
    seqlens = flat.reshape(B, S).sum(axis=1)
    pad = (-len(token_idx)) % pad_multiple if pad_multiple > 0 else 0
    if pad:
        seqlens = np.concatenate([seqlens, [pad]])
    cu = np.zeros(len(seqlens) + 1, dtype=np.int32)
    np.cumsum(seqlens, out=cu[1:])
    # packed index of every padded position (valid only where the mask is 1)
    packed_of = np.cumsum(flat, dtype=np.int32 if flat.size < 2**31 else np.int64) - 1
    # position p = S - R - 1 + t predicts response token t (dp_actor.py:236-237)
    t = np.arange(R)
    p = (S - R - 1) + t
    pos = (np.arange(B)[:, None] * S + p[None, :]).reshape(-1)
    nxt = pos + 1
    keep = flat[pos]  # real predictor: its log-prob is kept (0 where it is padding)
    sel_out = np.flatnonzero(keep)
    sel_hidden = packed_of[pos[keep]]
    label_idx = nxt[keep]
    tail = ~flat[nxt[keep]]  # last real token of a short row: label from the rolled packed stream
    if tail.any():
        first_real = np.argmax(attn_mask_cpu.astype(bool), axis=1)  # left-padded prompts
        bounds = np.asarray(groups if groups is not None else [0, B], dtype=np.int64)
        row = sel_out[tail] // R
        g = np.searchsorted(bounds, row, side="right") - 1
        nrow = row + 1
        wrap = nrow >= bounds[g + 1]
        nrow[wrap] = bounds[g[wrap]]
        label_idx[tail] = nrow * S + first_real[nrow]

    from ... import kernels as K

    # two host->device copies (one int64, one int32 buffer) instead of one per index array: the
    # plan is on the step's critical path before the first kernel; the tensors are views of them
    blocks, kblocks = attention.flash_block_table(cu), attention.flash_key_block_table(cu)
    i64 = [token_idx, sel_hidden, sel_out, label_idx, np.arange(pad)]
    i32 = [cu, blocks.reshape(-1), kblocks.reshape(-1)]
    d64 = K.h2d(np.concatenate(i64).astype(np.int64, copy=False), np.int64, device)
    d32 = K.h2d(np.concatenate(i32).astype(np.int32, copy=False), np.int32, device)

    def views(buf, parts):
        out, o = [], 0
        for a in parts:
            out.append(buf[o:o + len(a)])
            o += len(a)
        return out

    t_idx, s_hid, s_out, l_idx, p_pos = views(d64, i64)
    t_cu, t_blk, t_kblk = views(d32, i32)
    return _Packing(
        token_idx=t_idx,
        cu_seqlens=t_cu,
        max_seqlen=int(seqlens.max()) if B else 0,
        sel_hidden=s_hid,
        sel_out=s_out,
        label_idx=l_idx,
        attn_blocks=t_blk.view(-1, 2),
        attn_kblocks=t_kblk.view(-1, 2),
        pad=int(pad),
        pad_pos=p_pos if pad else None,
    )


def _scatter_rows(lp_sel, ent_sel, packing: _Packing, B: int, R: int, calculate_entropy: bool):
    """(entropy or None, log_probs) [B, R] from the selected rows' values (pad_input: 0 elsewhere)."""
    log_probs = lp_sel.new_zeros(B * R).index_copy(0, packing.sel_out, lp_sel).view(B, R)
    entropy = None
    if calculate_entropy:
        entropy = ent_sel.new_zeros(B * R).index_copy(0, packing.sel_out, ent_sel).view(B, R)
    return entropy, log_probs


def _mm_kwargs(multi_modal_inputs, device=None) -> dict:
    """dp_actor.py:94-98: the rows' multi-modal tensors concatenated along dim 0, on ``device``
    (the reference's FSDP module moves forward inputs to its device)."""
    if multi_modal_inputs is None or len(multi_modal_inputs) == 0:
        return {}
    return {k: torch.cat([d[k] for d in multi_modal_inputs], dim=0).to(device) for k in multi_modal_inputs[0]}


def hf_packed_hidden(backbone, ids: torch.Tensor, pos: torch.Tensor, packing: _Packing, multi_modal_inputs=None):
    """The HF backbone on one packed sequence (dp_actor.py:167-174: input_ids (1, nnz), position_ids
    (1, nnz) or (3, 1, nnz) for mrope, no attention mask, flash varlen via cu_seq_lens) -> [T, H]."""
    pos = pos.unsqueeze(0) if pos.dim() == 1 else pos.unsqueeze(1)
    inputs = dict(input_ids=ids.unsqueeze(0))
    if multi_modal_inputs:
        # the vision tower's outputs scattered over the placeholders here (qwen2_fused.input_embeddings),
        # so the packed-attention kwargs below reach the decoder only, never the vision tower
        from .qwen2_fused import input_embeddings

        inputs = dict(inputs_embeds=input_embeddings(backbone, ids, multi_modal_inputs).unsqueeze(0))
    out = backbone(
        **inputs, position_ids=pos, attention_mask=packed_mask_arg(backbone),
        use_cache=False, cu_seq_lens_q=packing.cu_seqlens, cu_seq_lens_k=packing.cu_seqlens,
        max_length_q=packing.max_seqlen, max_length_k=packing.max_seqlen,
    )
    return out.last_hidden_state[0]


def _multi_modal(mb: DataProto):
    """The micro-batch's multi_modal_inputs (non-tensor key, dp_actor.py:315-317), or None."""
    v = mb.non_tensor_batch.get("multi_modal_inputs") if mb.non_tensor_batch else None
    return None if v is None else list(v)


def merge_dynamic_passes(config, mini: DataProto, micro_batches: list, idx_lists: list, am, enabled: bool = True,
                         host_offsets: bool = False):
    """use_dynamic_bsz: consecutive token-budget micro-batches (in the reference's order,
    seqlen_balancing.rearrange_micro_batches) merged into update passes of at most
    ``config.compute_max_token_len_per_gpu`` tokens, for the actor and the critic. Returns (pass
    batches, their row index lists, per pass None or (int32 row offsets of its micro-batches on the
    device, device fp32 rows_s / ppo_mini_batch_size)). Without the key or with ``enabled`` False:
    the reference's micro-batches, one per pass. ``host_offsets``: also return, per pass, the host
    list of its micro-batches' row offsets (None for a single micro-batch)."""
    budget = config.get("compute_max_token_len_per_gpu", None)
    none = [None] * len(micro_batches)
    if not budget or not enabled or len(micro_batches) < 2:
        return (micro_batches, idx_lists, none, none) if host_offsets else (micro_batches, idx_lists, none)
    if am is None:  # padded path: no host copy yet (rearrange_micro_batches has synced already)
        am = mini.batch["attention_mask"].cpu().numpy()
    tokens = [int(am[np.asarray(ix, dtype=np.int64)].sum()) for ix in idx_lists]
    groups, cur, cur_tok = [], [], 0
    for j, t in enumerate(tokens):
        if cur and cur_tok + t > budget:
            groups.append(cur)
            cur, cur_tok = [], 0
        cur.append(j)
        cur_tok += t
    groups.append(cur)
    dev = mini.batch["input_ids"].device
    mini_rows = float(config.ppo_mini_batch_size)
    out_mb, out_idx, out_seg, out_host = [], [], [], []
    for g in groups:
        if len(g) == 1:
            out_mb.append(micro_batches[g[0]])
            out_idx.append(idx_lists[g[0]])
            out_seg.append(None)
            out_host.append(None)
            continue
        merged = [r for j in g for r in idx_lists[j]]
        rows = [len(idx_lists[j]) for j in g]
        offs = np.concatenate([[0], np.cumsum(rows)])
        out_mb.append(mini.select_idxs(np.asarray(merged, dtype=np.int64)))
        out_idx.append(merged)
        out_seg.append((K.seg_offsets(offs, dev, len(merged)),
                        K.h2d(np.asarray(rows, dtype=np.float32) / mini_rows, np.float32, dev)))
        out_host.append(offs.tolist())
    return (out_mb, out_idx, out_seg, out_host) if host_offsets else (out_mb, out_idx, out_seg)


class DataParallelPPOActor(BasePPOActor):
    def __init__(self, config, actor_module: nn.Module, actor_optimizer: torch.optim.Optimizer = None,
                 grad_reducer=None):
        """When actor_optimizer is None this is a reference policy (dp_actor.py:52-53)."""
        super().__init__(config)
        self.actor_module = actor_module
        self.actor_optimizer = actor_optimizer
        self.grad_reducer = grad_reducer
        self._am_cache = None  # (key, device mask, host copy): see _mask_host
        self.use_remove_padding = self.config.get("use_remove_padding", True)
        self.ulysses_sequence_parallel_size = self.config.get("ulysses_sequence_parallel_size", 1)
        if self.ulysses_sequence_parallel_size != 1:
            raise NotImplementedError("Ulysses sequence parallelism is out of scope for the DP actor-update path")
        base_prefix = getattr(actor_module, "base_model_prefix", "model")
        self._backbone = getattr(actor_module, base_prefix)
        self._lm_head = actor_module.get_output_embeddings()
        if self.use_remove_padding:
            attention.use_packed_attention(actor_module, self._backbone)
        self.device_name = "cuda"
        # bf16 autocast as the reference (dp_actor.py:100); None runs the model in its own dtype
        self.autocast_dtype = self.config.get("autocast_dtype", torch.bfloat16)
        # packed Qwen2 backbone with the fused add+RMSNorm / q|k|v+RoPE / SwiGLU kernels
        # (qwen2_fused.py; bf16 weights only, decided on first use)
        self.fused_model_ops = self.use_remove_padding and self.config.get("fused_model_ops", True)
        self._fused_backbone = None
        # fused lm_head + log-softmax + entropy (linear_logprob.hip): the
        # reference's use_fused_kernels flag turns it on for every pass (backward recomputes the
        # logits per chunk, dp_actor.py:163-190); fused_logprob_no_grad uses it only where no
        # gradient is needed (old / ref log-prob passes), where nothing has to be recomputed.
        self.use_fused_kernels = self.config.get("use_fused_kernels", False)
        # gfx950 flash-attention forward (attention.hip) inside the fused packed backbone
        self.fused_attention = self.config.get("fused_attention", True)
        self.fused_logprob_no_grad = self.config.get("fused_logprob_no_grad", False)
        # no-grad passes: gate|up GEMM + SwiGLU as one kernel (qwen2_fused.packed_forward fuse_mlp)
        self.fused_mlp_no_grad = bool(self.config.get("fused_mlp_no_grad", False))
        # update passes: the same kernel under autograd, also writing the projection for the backward
        self.fused_mlp_train = bool(self.config.get("fused_mlp_train", False))
        # all passes: the q|k|v GEMM + bias + RoPE as one kernel (qwen2_fused._qkv)
        self.fused_qkv = bool(self.config.get("fused_qkv", False))
        # no-grad passes with the fused lm_head: run all micro-batches' backbones, then the lm_head
        # launches back to back (compute_log_prob)
        self.fused_lm_head_after_backbone = bool(self.config.get("fused_lm_head_after_backbone", True))
        # ... in groups of micro-batches whose selected hidden states [n_sel, H] take at most this many
        # bytes together (each group's lm_heads run once its backbones have, and its hidden states are
        # freed then), so the pass holds a bounded amount beside the micro-batch being computed, as the
        # reference's log_prob_micro_batch_size bounds it; the bench's 4 x 131,072 x 896
        # bf16 rows (0.94 GB) are one group
        self.fused_lm_head_group_bytes = int(self.config.get("fused_lm_head_group_bytes", 2 << 30))
        # ... and as ONE launch over the concatenated rows
        self.fused_lm_head_concat = bool(self.config.get("fused_lm_head_concat", False))
        # the fused kernel's logits: bf16-rounded like the unfused autocast path and the reference's
        # default fused backend (fused_kernel_options.impl_backend "torch", ppo_trainer.yaml:91-94,
        # utils/experimental/torch_functional.py:20-37), or fp32 like its "triton" backend
        # (utils/kernel/kernels.py:120-346; fsdp_workers.py:298-309 selects it)
        fko = self.config.get("fused_kernel_options", None) or {}
        backend = fko.get("impl_backend", None) if hasattr(fko, "get") else None
        self.fused_kernel_fp32_logits = bool(self.config.get("fused_kernel_fp32_logits", backend == "triton"))
        # the log-prob backward writes dlogits over the logits (flash-attn inplace_backward, as the
        # reference) or into a fresh [N, V] buffer: on MI355X the out-of-place stream runs ~4 %
        # faster (a read+write pass whose writes hit other DRAM pages than its reads) for one more
        # logits-sized buffer at the backward's peak; "auto" takes the fresh buffer when the
        # allocator can provide it and the reference's in-place path when it cannot
        ipb = self.config.get("logprob_inplace_backward", True)
        self.logprob_inplace_backward = "auto" if ipb == "auto" else bool(ipb)
        # round packed micro-batches up to a multiple of this many tokens (0 = off) and look the
        # model GEMMs up in a tuned solution table (utils/gemm_tuning.py)
        self.pack_pad_multiple = int(self.config.get("pack_pad_multiple", 0) or 0)
        # backbone weight gradients + fp32 accumulation on a side stream beside the backward's
        # critical path (workers/grad_sync.MixedPrecisionParams.enable_wgrad_stream)
        self.wgrad_side_stream = bool(self.config.get("wgrad_side_stream", False))
        if (self.wgrad_side_stream and grad_reducer is not None
                and hasattr(grad_reducer, "enable_wgrad_stream")):
            # the decoder layers' weights: one gradient source each (not the tied lm_head / embedding)
            layers = getattr(self._backbone, "layers", None)
            self.wgrad_side_stream = layers is not None and grad_reducer.enable_wgrad_stream(
                list(layers.parameters()))
        else:
            self.wgrad_side_stream = False
        gemm_table = self.config.get("gemm_tuning_file", None)
        if gemm_table:
            from ...utils.gemm_tuning import use_tuned_gemms

            use_tuned_gemms(gemm_table)
        # rows per forward / backward pass of update_policy (None: ppo_micro_batch_size_per_gpu, the
        # reference). A multiple of ppo_micro_batch_size_per_gpu runs that many of the reference's
        # loss micro-batches in ONE pass: the fused loss kernel aggregates each micro-batch of
        # ppo_micro_batch_size_per_gpu rows on its own (seg_rows), so the loss, its gradient and the
        # per-micro-batch metric lists are the reference's (dp_actor.py:388-483) while the model
        # GEMMs see the larger token count.
        self.compute_micro_batch_size = self.config.get("compute_micro_batch_size_per_gpu", None)

    def _pass_rows(self, loss_mode: str) -> int:
        """Rows per update pass: compute_micro_batch_size_per_gpu rounded down to a multiple of
        ppo_micro_batch_size_per_gpu, where the fused vanilla loss can aggregate per micro-batch;
        the reference's micro-batch otherwise (registered loss variants draw their token selection
        per micro-batch, so they keep it)."""
        mb = int(self.config.ppo_micro_batch_size_per_gpu)
        cmb = self.compute_micro_batch_size
        if not cmb or loss_mode != "vanilla" or int(cmb) <= mb:
            return mb
        return int(cmb) // mb * mb


    # ------------------------------------------------------------------ forward
    def _forward_micro_batch(self, micro_batch, temperature, calculate_entropy=False, packing: _Packing = None,
                             multi_modal_inputs=None):
        """Returns (entropy or None, log_probs), both [bs, response_len] fp32. ``multi_modal_inputs``:
        the micro-batch's per-row dicts (non-tensor batch key of the same name, dp_actor.py:89-98)."""
        responses = micro_batch["responses"]
        R = responses.size(-1)
        input_ids = micro_batch["input_ids"]
        B, S = input_ids.shape
        ac = self.autocast_dtype
        with torch.autocast(device_type=self.device_name, dtype=ac or torch.bfloat16, enabled=ac is not None):
            if self.use_remove_padding:
                if packing is None:
                    packing = _plan_packing(micro_batch["attention_mask"].cpu().numpy(), R, input_ids.device,
                                            self.pack_pad_multiple)
                h_sel, labels = self._selected_hidden(micro_batch, packing, multi_modal_inputs)
                if self._use_fused_lm_head():
                    lp_sel, ent_sel = self._fused_lm_head_logprob(h_sel, labels, temperature)
                else:
                    head = self._lm_head
                    if (isinstance(head, nn.Linear) and head.bias is None and h_sel.is_cuda
                            and not (head._forward_hooks or head._forward_pre_hooks)):
                        # same forward GEMM; its input gradient runs over a transposed weight
                        # copy (kernels.input_grad: 32.1 -> 27.0 ms at 131,072 rows). A module
                        # with hooks is called as a module, so the hooks still fire.
                        logits = K.linear(h_sel, head.weight)
                    else:
                        logits = head(h_sel)
                    lp_sel, ent_sel = verl_F.logprobs_and_entropy_from_logits(
                        logits, labels, temperature, inplace_backward=self.logprob_inplace_backward)
                entropy, log_probs = _scatter_rows(lp_sel, ent_sel, packing, B, R, calculate_entropy)
            else:
                pos_ids = micro_batch["position_ids"]
                if pos_ids.dim() == 3:  # qwen2vl mrope (bsz, 3, seqlen) -> (3, bsz, seqlen), dp_actor.py:106-107
                    pos_ids = pos_ids.transpose(0, 1)
                out = self._backbone(
                    input_ids=input_ids, attention_mask=micro_batch["attention_mask"],
                    position_ids=pos_ids, use_cache=False, **_mm_kwargs(multi_modal_inputs, input_ids.device),
                )
                hidden = out.last_hidden_state[:, -R - 1 : -1]
                logits = self._lm_head(hidden)
                log_probs, ent = verl_F.logprobs_and_entropy_from_logits(
                    logits, responses, temperature, inplace_backward=self.logprob_inplace_backward)
                entropy = ent if calculate_entropy else None
        return entropy, log_probs

    def _selected_hidden(self, micro_batch, packing: _Packing, multi_modal_inputs=None):
        """The packed backbone over one micro-batch -> (hidden states of the rows whose log-prob is
        kept [n_sel, H], their labels [n_sel]) (dp_actor.py:167-190 up to the lm_head)."""
        input_ids = micro_batch["input_ids"]
        ids, pos = packing.gather(input_ids, micro_batch["position_ids"])
        if self._fused_backbone is None:
            from . import qwen2_fused

            self._fused_backbone = self.fused_model_ops and qwen2_fused.supports(self._backbone)
        if self._fused_backbone:
            from .qwen2_fused import packed_forward

            fa = self.fused_attention
            hidden = packed_forward(self._backbone, ids, pos, packing.cu_seqlens, packing.max_seqlen,
                                    attn_blocks=packing.attn_blocks if fa else None,
                                    attn_kblocks=packing.attn_kblocks if fa else None,
                                    multi_modal_inputs=multi_modal_inputs,
                                    fuse_mlp=self.fused_mlp_no_grad and not torch.is_grad_enabled(),
                                    fuse_mlp_train=self.fused_mlp_train, fuse_qkv=self.fused_qkv)
        else:
            hidden = hf_packed_hidden(self._backbone, ids, pos, packing, multi_modal_inputs)
        h_sel = hidden.index_select(0, packing.sel_hidden)
        labels = input_ids.reshape(-1).index_select(0, packing.label_idx)
        return h_sel, labels

    def _fused_lm_head_logprob(self, h_sel, labels, temperature, splits=None):
        w = self._lm_head.weight
        return K.linear_logprob_entropy(h_sel.to(torch.bfloat16), w if w.dtype == torch.bfloat16 else w.to(torch.bfloat16),
                                        labels, temperature, fp32_logits=self.fused_kernel_fp32_logits, splits=splits)

    def _fused_lm_head_group(self, group: list, temperature, calculate_entropy: bool, lps: list, ents: list):
        """The fused lm_head launches of a group of micro-batches whose backbones have run (``group``
        = [(micro-batch, plan, h_sel, labels)], emptied here: each h_sel is released once its launch
        is queued), back to back, or as one launch over the concatenated rows (fused_lm_head_concat,
        with the vocab ranges a micro-batch's own launch would use: the same per-row bits for
        equal-sized micro-batches); per-response log-probs / entropies appended to lps / ents."""
        if self.fused_lm_head_concat and len(group) > 1:
            sizes = [g[2].shape[0] for g in group]
            lp_all, ent_all = self._fused_lm_head_logprob(
                torch.cat([g[2] for g in group]), torch.cat([g[3] for g in group]), temperature,
                splits=K._linear_logprob_splits(max(sizes)))
            outs = list(zip(lp_all.split(sizes), ent_all.split(sizes), strict=True))
            for g in group:
                g[2] = None
        else:
            outs = []
            for g in group:
                outs.append(self._fused_lm_head_logprob(g[2], g[3], temperature))
                g[2] = None
        for (mb, plan, _, _), (lp_sel, ent_sel) in zip(group, outs, strict=True):
            B, R = mb.batch["responses"].shape
            ent, lp = _scatter_rows(lp_sel, ent_sel, plan, B, R, calculate_entropy)
            lps.append(lp)
            if calculate_entropy:
                ents.append(ent)
        group.clear()

    def _use_fused_lm_head(self) -> bool:
        head = self._lm_head
        if not isinstance(head, nn.Linear) or head.bias is not None:
            return False
        return bool(self.use_fused_kernels or (self.fused_logprob_no_grad and not torch.is_grad_enabled()))

    def _mask_host(self, am_t: torch.Tensor, refresh: bool = False) -> np.ndarray:
        """Host copy of the attention mask, which plans padding removal. A device->host copy drains
        the stream: at the start of a step it would leave the GPU idle while the host plans, and at
        the start of the update it would wait for the queued old-logp pass and advantage work. So,
        in this order:
          * the host copy DataProto.to took of a host batch's mask (protocol.HOST_MIRRORED_KEY: a
            clone only it holds), while the device tensor has not been written since;
          * the copy taken last, while the tensor is the same unmodified one (same storage, shape
            and in-place version: the step's compute_log_prob and update_policy, or the same batch
            again);
          * else one device->host copy (also with ``refresh``).

        Contract: the mask must not change other than through ordinary in-place tensor writes
        (which bump the version); writes through ``.data`` or through another tensor sharing the
        storage are not seen and would leave the passes planned from the stale copy. The step
        driver (trainer_step.PPOTrainerStep) never writes the mask."""
        # the cache holds the device tensor itself, so its storage cannot be freed and reused by
        # another batch's mask while the key (pointer, shape, in-place version) is compared
        key = (am_t.data_ptr(), tuple(am_t.shape), am_t._version, am_t.device)
        if not refresh and self._am_cache is not None and self._am_cache[0] == key:
            return self._am_cache[2]
        mirror = getattr(am_t, "_va_host_mirror", None)
        if (not refresh and mirror is not None and am_t._version == mirror[1]
                and tuple(mirror[0].shape) == tuple(am_t.shape)):
            am = mirror[0].numpy()
        else:
            am = am_t.cpu().numpy()
        self._am_cache = (key, am_t, am)
        return am

    def _plans(self, data: DataProto, sizes: list[int] = None, idx_lists: list[list[int]] = None,
               am: np.ndarray = None, group_rows: int = 0, groups: list = None) -> list:
        """Packing plans of consecutive micro-batches of ``sizes`` rows, or of the dynamic
        micro-batches' row index lists, from one host copy of the attention mask. The reference's
        micro-batches inside each: runs of ``group_rows`` rows, or per plan the row offsets in
        ``groups`` (None: the micro-batch itself)."""
        n_mb = len(sizes) if idx_lists is None else len(idx_lists)
        if not self.use_remove_padding:
            return [None] * n_mb
        if am is None:
            am = data.batch["attention_mask"].cpu().numpy()
        R = data.batch["responses"].size(-1)
        dev = data.batch["input_ids"].device
        if groups is None:
            groups = [None] * n_mb
        if idx_lists is not None:
            return [_plan_packing(am[np.asarray(ix, dtype=np.int64)], R, dev, self.pack_pad_multiple, g)
                    for ix, g in zip(idx_lists, groups, strict=True)]
        plans, s = [], 0
        for n, g in zip(sizes, groups, strict=True):
            if g is None and group_rows and n > group_rows:
                g = list(range(0, n, group_rows)) + [n]
            plans.append(_plan_packing(am[s : s + n], R, dev, self.pack_pad_multiple, g))
            s += n
        return plans

    # ------------------------------------------------------------------ optimizer
    def _zero_grad(self):
        if self.grad_reducer is not None:
            self.grad_reducer.zero_grad()
        else:
            self.actor_optimizer.zero_grad()

    def _optimizer_step(self):
        assert self.config.grad_clip is not None
        if self.grad_reducer is not None:
            self.grad_reducer.finish_sync()
        grad_norm = clip_grad_norm(self.grad_reducer, self.actor_module, self.config.grad_clip)
        return step_unless_nonfinite(self.actor_optimizer, grad_norm, self._zero_grad,
                                     self.grad_reducer.after_step if self.grad_reducer is not None else None)

    # ------------------------------------------------------------------ API
    @torch.no_grad()
    def compute_log_prob(self, data: DataProto, calculate_entropy=False):
        """dp_actor.py:290-349 — old-logp (and entropy) over micro-batches, no grad."""
        self.actor_module.eval()
        micro_batch_size = data.meta_info["micro_batch_size"]
        temperature = data.meta_info["temperature"]
        use_dynamic_bsz = data.meta_info["use_dynamic_bsz"]
        has_mm = "multi_modal_inputs" in data.non_tensor_batch.keys()
        data = data.select(batch_keys=["responses", "input_ids", "attention_mask", "position_ids"],
                           non_tensor_batch_keys=["multi_modal_inputs"] if has_mm else [])
        am = (self._mask_host(data.batch["attention_mask"], refresh=BLOCKING_STEP_BOUNDARY)
              if self.use_remove_padding else None)
        if use_dynamic_bsz:
            # dp_actor.py:321-323: micro-batches cut by a token budget, restored afterwards
            max_token_len = data.meta_info["max_token_len"] * self.ulysses_sequence_parallel_size
            micro_batches, batch_idx_list = prepare_dynamic_batch(data, max_token_len=max_token_len)
            plans = self._plans(data, idx_lists=batch_idx_list, am=am)
        else:
            micro_batches = data.split(micro_batch_size)
            plans = self._plans(data, [len(m) for m in micro_batches], am=am)
        lps, ents = [], []
        if self.use_remove_padding and self._use_fused_lm_head() and self.fused_lm_head_after_backbone:
            # every micro-batch's backbone first, then their fused lm_head launches back to back: f1
            # right after the backbone's power-capped GEMMs starts clocked down (33.1 ms alone, 34.9 ms
            # right after GEMM load, 33.4 ms per launch over 4 in a row; profiles/r05/f1_pre_gemm_load.jsonl),
            # so consecutive launches recover the clock. Per-row results are the same bits.
            with torch.autocast(device_type=self.device_name, dtype=self.autocast_dtype or torch.bfloat16,
                                enabled=self.autocast_dtype is not None):
                group, held = [], 0
                for i, (mb, plan) in enumerate(zip(micro_batches, plans, strict=True)):
                    h_sel, labels = self._selected_hidden(mb.batch, plan, _multi_modal(mb))
                    held += h_sel.numel() * h_sel.element_size()
                    group.append([mb, plan, h_sel, labels])
                    h_sel = labels = None
                    if held >= self.fused_lm_head_group_bytes or i == len(micro_batches) - 1:
                        self._fused_lm_head_group(group, temperature, calculate_entropy, lps, ents)
                        group, held = [], 0
        else:
            for mb, plan in zip(micro_batches, plans, strict=True):
                ent, lp = self._forward_micro_batch(mb.batch, temperature, calculate_entropy, plan, _multi_modal(mb))
                lps.append(lp)
                if calculate_entropy:
                    ents.append(ent)
        log_probs = torch.concat(lps, dim=0)
        entropys = torch.concat(ents, dim=0) if calculate_entropy else None
        if use_dynamic_bsz:
            log_probs = restore_dynamic_batch(log_probs, batch_idx_list)
            if entropys is not None:
                entropys = restore_dynamic_batch(entropys, batch_idx_list)
        return log_probs, entropys

    def update_policy(self, data: DataProto):
        """dp_actor.py:351-486 — PPO epochs x mini-batches x micro-batches; one optimizer step per
        mini-batch; returns {metric: [values]}."""
        self.actor_module.train()
        temperature = data.meta_info["temperature"]
        cfg = self.config
        keys = ["responses", "response_mask", "input_ids", "attention_mask", "position_ids", "old_log_probs",
                "advantages"]
        if cfg.use_kl_loss:
            keys.append("ref_log_prob")
        has_mm = "multi_modal_inputs" in data.non_tensor_batch.keys()
        data = data.select(batch_keys=keys, non_tensor_batch_keys=["multi_modal_inputs"] if has_mm else [])
        am_full = self._mask_host(data.batch["attention_mask"]) if self.use_remove_padding else None
        mini_batches = data.split(cfg.ppo_mini_batch_size)
        if not cfg.use_dynamic_bsz:
            self.gradient_accumulation = cfg.ppo_mini_batch_size // cfg.ppo_micro_batch_size_per_gpu
        clip_ratio = cfg.clip_ratio
        clip_low = cfg.clip_ratio_low if cfg.get("clip_ratio_low") is not None else clip_ratio
        clip_high = cfg.clip_ratio_high if cfg.get("clip_ratio_high") is not None else clip_ratio
        clip_c = cfg.get("clip_ratio_c", 3.0)
        entropy_coeff = cfg.entropy_coeff
        agg_mode = cfg.loss_agg_mode
        loss_mode = cfg.policy_loss.get("loss_mode", "vanilla")

        dev_metrics: dict[str, list] = {}
        for _ in range(cfg.ppo_epochs):
            row0 = 0
            for mini in mini_batches:
                am = am_full[row0 : row0 + len(mini)] if am_full is not None else None  # split keeps row order
                row0 += len(mini)
                if cfg.use_dynamic_bsz:
                    # dp_actor.py:382-384
                    max_token_len = cfg.ppo_max_token_len_per_gpu * self.ulysses_sequence_parallel_size
                    micro_batches, idx_lists = prepare_dynamic_batch(mini, max_token_len=max_token_len)
                    # registered loss variants draw their token selection per micro-batch: never merged
                    micro_batches, idx_lists, seg_offs, seg_rows_h = merge_dynamic_passes(
                        cfg, mini, micro_batches, idx_lists, am, loss_mode == "vanilla", host_offsets=True)
                    plans = self._plans(mini, idx_lists=idx_lists, am=am, groups=seg_rows_h)
                else:
                    seg_mb = int(cfg.ppo_micro_batch_size_per_gpu)
                    micro_batches = mini.split(self._pass_rows(loss_mode))
                    plans = self._plans(mini, [len(m) for m in micro_batches], am=am, group_rows=seg_mb)
                    seg_offs = [None] * len(micro_batches)
                self._zero_grad()
                for i, (mb, plan, seg_off) in enumerate(zip(micro_batches, plans, seg_offs, strict=True)):
                    b = mb.batch
                    response_mask = b["response_mask"]
                    calc_ent = entropy_coeff != 0
                    entropy, log_prob = self._forward_micro_batch(b, temperature, calc_ent, plan, _multi_modal(mb))
                    m = {}
                    # several of the reference's loss micro-batches in this pass: aggregated one by one
                    # (uniform runs of seg_mb rows, or the token-budget micro-batches' row ranges seg_off)
                    seg = seg_mb if not cfg.use_dynamic_bsz and len(mb) > seg_mb else 0
                    if loss_mode == "vanilla":
                        out = core_algos.compute_actor_loss(
                            b["old_log_probs"], log_prob, b["advantages"], response_mask, clip_low, clip_high,
                            clip_c, agg_mode, entropy=entropy if calc_ent else None,
                            ref_log_prob=b["ref_log_prob"] if cfg.use_kl_loss else None,
                            kl_loss_type=cfg.kl_loss_type if cfg.use_kl_loss else None, seg_rows=seg,
                            seg_off=None if seg_off is None else seg_off[0],
                        )
                        # [8] or [S, 8]: the slots below are scalars or one value per loss micro-batch
                        pg_loss, pg_clipfrac = out[..., L.VA_LOSS_PG], out[..., L.VA_LOSS_CLIPFRAC]
                        ppo_kl, pg_clipfrac_lower = out[..., L.VA_LOSS_PPO_KL], out[..., L.VA_LOSS_CLIPFRAC_LOWER]
                        policy_loss = pg_loss
                        if calc_ent:
                            policy_loss = pg_loss - out[..., L.VA_LOSS_ENTROPY] * entropy_coeff
                        if cfg.use_kl_loss:
                            kl_loss = out[..., L.VA_LOSS_KL]
                            policy_loss = policy_loss + kl_loss * cfg.kl_loss_coef
                            m["actor/kl_loss"] = kl_loss.detach()
                            m["actor/kl_coef"] = cfg.kl_loss_coef
                    else:
                        fn = get_policy_loss_fn(loss_mode)
                        pg_loss, pg_clipfrac, ppo_kl, pg_clipfrac_lower = fn(
                            old_log_prob=b["old_log_probs"], log_prob=log_prob, advantages=b["advantages"],
                            response_mask=response_mask, loss_agg_mode=agg_mode, config=cfg)
                        policy_loss = pg_loss
                        if calc_ent:
                            policy_loss = pg_loss - agg_loss(entropy, response_mask, agg_mode) * entropy_coeff
                        if cfg.use_kl_loss:
                            kld = kl_penalty(log_prob, b["ref_log_prob"], cfg.kl_loss_type)
                            kl_loss = agg_loss(kld, response_mask, agg_mode)
                            policy_loss = policy_loss + kl_loss * cfg.kl_loss_coef
                            m["actor/kl_loss"] = kl_loss.detach()
                            m["actor/kl_coef"] = cfg.kl_loss_coef
                    if cfg.use_dynamic_bsz and seg_off is not None:
                        # each micro-batch's loss relative to the dynamic bsz: sum_s policy_loss_s * rows_s / mini
                        loss = (policy_loss * seg_off[1]).sum()
                    elif cfg.use_dynamic_bsz:
                        # relative to the dynamic bsz (dp_actor.py:465-467)
                        loss = policy_loss * (response_mask.shape[0] / cfg.ppo_mini_batch_size)
                    elif seg:
                        # sum over the pass's micro-batches of policy_loss / gradient_accumulation: the
                        # gradient the reference accumulates over their separate backward passes
                        loss = (policy_loss / self.gradient_accumulation).sum()
                    else:
                        loss = policy_loss / self.gradient_accumulation
                    last = i == len(micro_batches) - 1
                    if last and self.grad_reducer is not None:
                        self.grad_reducer.begin_sync()
                    if self.wgrad_side_stream:
                        K.WGRAD_SINK = self.grad_reducer
                    try:
                        loss.backward()
                    finally:
                        K.WGRAD_SINK = None
                    if self.grad_reducer is not None:
                        self.grad_reducer.after_backward()
                    m.update({
                        "actor/pg_loss": pg_loss.detach(),
                        "actor/pg_clipfrac": pg_clipfrac.detach(),
                        "actor/ppo_kl": ppo_kl.detach(),
                        "actor/pg_clipfrac_lower": pg_clipfrac_lower.detach(),
                    })
                    if seg or seg_off is not None:  # one entry per loss micro-batch, in order (the reference's)
                        for k in range(pg_loss.shape[0]):
                            append_to_dict(dev_metrics, {
                                key: (v[k] if isinstance(v, torch.Tensor) else v) for key, v in m.items()})
                    else:
                        append_to_dict(dev_metrics, m)
                grad_norm = self._optimizer_step()
                append_to_dict(dev_metrics, {"actor/grad_norm": grad_norm.detach()})
        self._zero_grad()
        return _to_host(dev_metrics)


# VERL_AMD_TORCH_CLIP=1: torch.nn.utils.clip_grad_norm_ over the masters even when the parameter
# manager has its bucket clip (A/B runs; the sharded manager always uses its own)
_TORCH_CLIP = os.environ.get("VERL_AMD_TORCH_CLIP", "0") == "1"


def clip_grad_norm(grad_reducer, module: nn.Module, max_norm: float) -> torch.Tensor:
    """Global gradient-norm clip of the actor or critic (dp_actor.py:272-280, dp_critic.py:138-146):
    the parameter manager's own clip (fsdp_utils.py:503-516) over its flat fp32 buckets, or the
    global norm over the ranks' shards for the sharded optimizer state; torch's clip_grad_norm_
    over the masters without a manager or with VERL_AMD_TORCH_CLIP=1 (replicated managers only)."""
    if (grad_reducer is not None and hasattr(grad_reducer, "clip_grad_norm_")
            and not (_TORCH_CLIP and not hasattr(grad_reducer, "shards"))):
        return grad_reducer.clip_grad_norm_(max_norm)
    params = grad_reducer.optimizer_params() if grad_reducer is not None else list(module.parameters())
    return torch.nn.utils.clip_grad_norm_(params, max_norm=max_norm, foreach=True)


def step_unless_nonfinite(optimizer, grad_norm: torch.Tensor, zero_grad, after_step=None):
    """dp_actor.py:272-288: step unless the clipped-gradient norm is not finite (then warn and
    drop the gradients). A fused device optimizer skips the step ON the device (its found_inf
    input, the GradScaler mechanism: parameters, moments and step counts untouched), so the
    update needs no host sync here; the warning is printed when the metrics reach the host
    (``_to_host`` sees the non-finite grad_norm) and the dropped gradients are zeroed by the
    next mini-batch's zero_grad as in the reference. Other optimizers keep the host check."""
    fused = bool(optimizer.defaults.get("fused")) and grad_norm.is_cuda
    if fused:
        optimizer.found_inf = (~torch.isfinite(grad_norm)).to(torch.float32).reshape(())  # 0-d, as the step counts
        try:
            optimizer.step()
        finally:
            optimizer.found_inf = None
        if after_step is not None:
            after_step()  # re-derives the compute weights from unchanged masters when skipped
        return grad_norm
    if not torch.isfinite(grad_norm):
        rank = torch.distributed.get_rank() if torch.distributed.is_initialized() else 0
        print(f"WARN: rank {rank} grad_norm is not finite: {grad_norm}")
        zero_grad()
    else:
        optimizer.step()
        if after_step is not None:
            after_step()
    return grad_norm


class DeviceMetrics(MutableMapping):
    """The metric lists of one update, read back without blocking the host (the reference calls
    .item() per micro-batch, dp_actor.py:462-483, a host sync each): every device value goes into
    ONE pinned host buffer by an asynchronous copy at the end of the update, and the first read
    waits for that copy's event. Until then the host runs on — into the next step's planning
    while the GPU finishes the optimizer step — so the GPU is not left idle at the step boundary.
    Host values (e.g. kl_coef) never go to the device. Keys set before the first read are kept;
    ``on_ready`` callbacks (e.g. the update's MFU from its device time) run once, after the copy."""

    def __init__(self, dev_metrics: dict, on_ready=()):
        dev_keys, dev_vals, out_pos = [], [], []
        out: dict[str, list] = {}
        for k, lst in dev_metrics.items():
            if not isinstance(lst, (list, tuple)):  # a scalar entry stays as it is
                out[k] = lst.item() if isinstance(lst, torch.Tensor) else lst
                continue
            dst = out.setdefault(k, [])
            for v in lst:
                if isinstance(v, torch.Tensor):
                    dev_keys.append(k)
                    out_pos.append(len(dst))
                    dev_vals.append(v.detach().float().reshape(()))
                    dst.append(None)
                else:
                    dst.append(float(v))
        self._data = out
        self._slots = list(zip(dev_keys, out_pos, strict=True))
        self._host = self._event = None
        self._on_ready = list(on_ready)
        if dev_vals:
            devs = {v.device for v in dev_vals}
            if len(devs) == 1 and dev_vals[0].is_cuda:
                flat = torch.stack(dev_vals)
                self._host = torch.empty(flat.shape, dtype=flat.dtype, pin_memory=True)
                self._host.copy_(flat, non_blocking=True)
                self._event = torch.cuda.Event()
                self._event.record(torch.cuda.current_stream(flat.device))
            else:  # host tensors, or several devices: read now
                self._host = torch.stack([v.cpu() for v in dev_vals])
        if self._host is None:
            self._finish()

    def add_on_ready(self, fn):
        """Run ``fn(self)`` once the device values are in (now, if they already are)."""
        if self._slots is None:
            fn(self)
        else:
            self._on_ready.append(fn)

    def _finish(self):
        if self._slots is None:
            return
        if self._event is not None:
            self._event.synchronize()
        if self._host is not None:
            for (k, i), v in zip(self._slots, self._host.tolist(), strict=True):
                self._data[k][i] = v
        self._slots, self._host, self._event = None, None, None
        for k, lst in self._data.items():
            if k.endswith("grad_norm") and isinstance(lst, list) and not all(np.isfinite(g) for g in lst):
                rank = torch.distributed.get_rank() if torch.distributed.is_initialized() else 0
                print(f"WARN: rank {rank} {k} is not finite: {lst} (optimizer step skipped)")
        fns, self._on_ready = self._on_ready, []
        for fn in fns:
            fn(self)

    def __getitem__(self, k):
        self._finish()
        return self._data[k]

    def __setitem__(self, k, v):
        self._data[k] = v

    def __delitem__(self, k):
        self._finish()
        del self._data[k]

    def __iter__(self):
        self._finish()
        return iter(dict(self._data))

    def __len__(self):
        self._finish()
        return len(self._data)

    def __repr__(self):
        self._finish()
        return f"DeviceMetrics({self._data!r})"

    def __reduce__(self):
        # pickled (e.g. in a DataProto's meta_info across a process boundary) as the plain dict of
        # host values: the pinned buffer and the event stay behind
        self._finish()
        return (dict, (dict(self._data),))


# VERL_AMD_BLOCKING_STEP_BOUNDARY=1 restores the round-4 step boundary for A/B runs: the update's
# metrics are read back before update_policy returns (a host sync), and compute_log_prob always
# copies the attention mask device->host
BLOCKING_STEP_BOUNDARY = os.environ.get("VERL_AMD_BLOCKING_STEP_BOUNDARY", "0") == "1"


def _to_host(dev_metrics: dict) -> DeviceMetrics:
    """The update's metrics as a DeviceMetrics (one asynchronous device->host copy)."""
    m = DeviceMetrics(dev_metrics)
    if BLOCKING_STEP_BOUNDARY:
        len(m)  # waits for the copy here
    return m
