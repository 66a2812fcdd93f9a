"""DataParallelPPOCritic — mirror of verl/workers/critic/dp_critic.py:46-256 on MI355X
(the critic of config 3, PPO with GAE).

Same constructor, config keys, micro/mini-batch loops (fixed or token-budget dynamic), loss
scaling and metric keys as the reference. The hot path maps onto the GPU like the actor's:

  * padding removal planned once per call on the host (one D2H of the attention mask); the
    backbone runs on packed tokens (qwen2_fused.packed_forward for bf16 Qwen2: fused
    add+RMSNorm, merged q|k|v + RoPE, merged gate|up + SwiGLU, flash varlen attention);
  * only the hidden states at positions that predict a response token go through the value
    head (the reference scores every token and slices :, -R-1:-1 afterwards, dp_critic.py:123-124);
  * the clipped value loss, vf_clipfrac and vpred_mean are ONE fused kernel pair
    (va_value_loss_fwd/bwd); metrics stay on device until one transfer per update;
  * gradients go through the same bucketed RCCL reducer / fp32-master manager as the actor.
Values are returned in fp32 (the reference's bf16 autocast values, upcast exactly; GAE promotes
them to fp32 anyway, core_algos.py:225-230).
"""

from __future__ import annotations

import torch
from torch import nn

from ... import _lib as L
from ... import kernels as K
from ...protocol import DataProto
from ...utils.seqlen_balancing import prepare_dynamic_batch, restore_dynamic_batch
from ..actor import attention
from ..actor.dp_actor import (_mm_kwargs, _multi_modal, _plan_packing, _to_host, append_to_dict, clip_grad_norm,
                              hf_packed_hidden, merge_dynamic_passes, step_unless_nonfinite)
from .base import BasePPOCritic

__all__ = ["DataParallelPPOCritic"]


class DataParallelPPOCritic(BasePPOCritic):
    def __init__(self, config, critic_module: nn.Module, critic_optimizer: torch.optim.Optimizer, grad_reducer=None):
        super().__init__(config=config)
        self.critic_module = critic_module
        self.critic_optimizer = critic_optimizer
        self.grad_reducer = grad_reducer
        model_cfg = self.config.get("model", {}) or {}
        self.use_remove_padding = model_cfg.get("use_remove_padding", False)
        self.ulysses_sequence_parallel_size = self.config.get("ulysses_sequence_parallel_size", 1)
        if self.ulysses_sequence_parallel_size != 1:
            raise NotImplementedError("Ulysses sequence parallelism is out of scope for the DP critic path")
        self.device_name = "cuda"
        prefix = getattr(critic_module, "base_model_prefix", "model")
        self._backbone = getattr(critic_module, prefix)
        self._head = getattr(critic_module, "score", None)
        if self._head is None:
            raise NotImplementedError("critic needs a token-classification value head (.score, num_labels=1)")
        if self.use_remove_padding:
            attention.use_packed_attention(critic_module, self._backbone)
        self.fused_model_ops = self.use_remove_padding and self.config.get("fused_model_ops", True)
        self._fused_backbone = None
        # as the actor: pad packed micro-batches to a multiple of this many tokens (0 = off) and
        # use a tuned GEMM solution table
        self.pack_pad_multiple = int(self.config.get("pack_pad_multiple", 0) or 0)
        if self.config.get("gemm_tuning_file", None):
            from ...utils.gemm_tuning import use_tuned_gemms

            use_tuned_gemms(self.config.gemm_tuning_file)
        # as the actor: rows per update pass, a multiple of ppo_micro_batch_size_per_gpu whose loss
        # micro-batches the fused value loss aggregates one by one (None: the reference's micro-batch)
        self.compute_micro_batch_size = self.config.get("compute_micro_batch_size_per_gpu", None)

    def _pass_rows(self) -> int:
        mb = int(self.config.ppo_micro_batch_size_per_gpu)
        cmb = self.compute_micro_batch_size
        return int(cmb) // mb * mb if cmb and int(cmb) > mb else mb

    # ------------------------------------------------------------------ forward
    def _forward_micro_batch(self, micro_batch, packing=None, multi_modal_inputs=None) -> torch.Tensor:
        """values [bs, response_len] fp32 (dp_critic.py:57-136); mrope position ids [bs, 3, S] and
        multi_modal_inputs as the actor (dp_critic.py:59-90)."""
        R = micro_batch["responses"].size(-1)
        input_ids = micro_batch["input_ids"]
        B, S = input_ids.shape
        position_ids = micro_batch["position_ids"]
        with torch.autocast(device_type=self.device_name, dtype=torch.bfloat16):
            if self.use_remove_padding:
                if packing is None:
                    packing = _plan_packing(micro_batch["attention_mask"].cpu().numpy(), R, input_ids.device,
                                            self.pack_pad_multiple)
                ids, pos = packing.gather(input_ids, position_ids)
                if self._fused_backbone is None:
                    from ..actor import qwen2_fused

                    self._fused_backbone = self.fused_model_ops and qwen2_fused.supports(self._backbone)
                if self._fused_backbone:
                    from ..actor.qwen2_fused import packed_forward

                    fa = self.config.get("fused_attention", True)
                    hidden = packed_forward(self._backbone, ids, pos, packing.cu_seqlens, packing.max_seqlen,
                                            attn_blocks=packing.attn_blocks if fa else None,
                                            attn_kblocks=packing.attn_kblocks if fa else None,
                                            multi_modal_inputs=multi_modal_inputs)
                else:
                    hidden = hf_packed_hidden(self._backbone, ids, pos, packing, multi_modal_inputs)
                v_sel = self._head(hidden.index_select(0, packing.sel_hidden)).squeeze(-1).float()
                values = v_sel.new_zeros(B * R).index_copy(0, packing.sel_out, v_sel).view(B, R)
            else:
                if position_ids.dim() == 3:  # qwen2vl mrope (dp_critic.py:71-72)
                    position_ids = position_ids.transpose(0, 1)
                out = self.critic_module(input_ids=input_ids, attention_mask=micro_batch["attention_mask"],
                                         position_ids=position_ids, use_cache=False,
                                         **_mm_kwargs(multi_modal_inputs, input_ids.device))
                values = out.logits[:, -R - 1 : -1].squeeze(-1).float()
        return values

    def _plans(self, data: DataProto, sizes=None, idx_lists=None):
        n_mb = len(sizes) if idx_lists is None else len(idx_lists)
        if not self.use_remove_padding:
            return [None] * n_mb
        import numpy as np

        am = data.batch["attention_mask"].cpu().numpy()
        R = data.batch["responses"].size(-1)
        dev = data.batch["input_ids"].device
        if idx_lists is not None:
            return [_plan_packing(am[np.asarray(ix, dtype=np.int64)], R, dev, self.pack_pad_multiple)
                    for ix in idx_lists]
        plans, s = [], 0
        for n in sizes:
            plans.append(_plan_packing(am[s : s + n], R, dev, self.pack_pad_multiple))
            s += n
        return plans

    # ------------------------------------------------------------------ optimizer
    def _zero_grad(self):
        if self.grad_reducer is not None:
            self.grad_reducer.zero_grad()
        else:
            self.critic_optimizer.zero_grad()

    def _optimizer_step(self):
        """dp_critic.py:138-154."""
        assert self.config.grad_clip is not None
        if self.grad_reducer is not None:
            self.grad_reducer.finish_sync()
        grad_norm = clip_grad_norm(self.grad_reducer, self.critic_module, self.config.grad_clip)
        return step_unless_nonfinite(self.critic_optimizer, grad_norm, self._zero_grad,
                                     self.grad_reducer.after_step if self.grad_reducer is not None else None)

    # ------------------------------------------------------------------ API
    @torch.no_grad()
    def compute_values(self, data: DataProto) -> torch.Tensor:
        """dp_critic.py:156-191 — values over micro-batches, masked by response_mask."""
        self.critic_module.eval()
        micro_batch_size = data.meta_info["micro_batch_size"]
        use_dynamic_bsz = data.meta_info["use_dynamic_bsz"]
        has_mm = "multi_modal_inputs" in data.non_tensor_batch.keys()
        data = data.select(batch_keys=["responses", "input_ids", "response_mask", "attention_mask", "position_ids"],
                           non_tensor_batch_keys=["multi_modal_inputs"] if has_mm else [])
        if use_dynamic_bsz:
            max_token_len = data.meta_info["max_token_len"] * self.ulysses_sequence_parallel_size
            micro_batches, batch_idx_list = prepare_dynamic_batch(data, max_token_len=max_token_len)
            plans = self._plans(data, idx_lists=batch_idx_list)
        else:
            micro_batches = data.split(micro_batch_size)
            plans = self._plans(data, [len(m) for m in micro_batches])
        vals = [self._forward_micro_batch(mb.batch, plan, _multi_modal(mb))
                for mb, plan in zip(micro_batches, plans, strict=True)]
        values = torch.concat(vals, dim=0)
        if use_dynamic_bsz:
            values = restore_dynamic_batch(values, batch_idx_list)
        return values * data.batch["response_mask"]  # only action tokens have values

    def update_critic(self, data: DataProto):
        """dp_critic.py:193-256 — PPO epochs x mini-batches x micro-batches of the clipped value
        loss; one optimizer step per mini-batch; returns {metric: [values]}."""
        self.critic_module.train()
        cfg = self.config
        keys = ["input_ids", "responses", "response_mask", "attention_mask", "position_ids", "values", "returns"]
        has_mm = "multi_modal_inputs" in data.non_tensor_batch.keys()
        data = data.select(batch_keys=keys, non_tensor_batch_keys=["multi_modal_inputs"] if has_mm else [])
        mini_batches = data.split(cfg.ppo_mini_batch_size)
        dev_metrics: dict = {}
        for _ in range(cfg.ppo_epochs):
            for mini in mini_batches:
                if cfg.use_dynamic_bsz:
                    max_token_len = cfg.ppo_max_token_len_per_gpu * self.ulysses_sequence_parallel_size
                    micro_batches, idx_lists = prepare_dynamic_batch(mini, max_token_len=max_token_len)
                    micro_batches, idx_lists, seg_offs = merge_dynamic_passes(cfg, mini, micro_batches, idx_lists,
                                                                              None)
                    plans = self._plans(mini, idx_lists=idx_lists)
                else:
                    self.gradient_accumulation = cfg.ppo_mini_batch_size // cfg.ppo_micro_batch_size_per_gpu
                    micro_batches = mini.split(self._pass_rows())
                    plans = self._plans(mini, [len(m) for m in micro_batches])
                    seg_offs = [None] * len(micro_batches)
                self._zero_grad()
                for i, (mb, plan, seg_off) in enumerate(zip(micro_batches, plans, seg_offs, strict=True)):
                    b = mb.batch
                    response_mask = b["response_mask"]
                    vpreds = self._forward_micro_batch(b, plan, _multi_modal(mb))
                    # several of the reference's loss micro-batches in this pass: aggregated one by one
                    seg = (int(cfg.ppo_micro_batch_size_per_gpu)
                           if not cfg.use_dynamic_bsz and len(mb) > int(cfg.ppo_micro_batch_size_per_gpu) else 0)
                    out = K.fused_value_loss(vpreds, b["values"], b["returns"], response_mask, cfg.cliprange_value,
                                             cfg.loss_agg_mode, seg_rows=seg,
                                             seg_off=None if seg_off is None else seg_off[0])
                    vf_loss = out[..., L.VA_VLOSS_LOSS]  # scalar, or one value per loss micro-batch
                    if cfg.use_dynamic_bsz and seg_off is not None:
                        loss = (vf_loss * seg_off[1]).sum()  # sum_s vf_loss_s * rows_s / mini (dp_critic.py:226)
                    elif cfg.use_dynamic_bsz:
                        loss = vf_loss * (response_mask.shape[0] / cfg.ppo_mini_batch_size)
                    elif seg:
                        loss = (vf_loss / self.gradient_accumulation).sum()
                    else:
                        loss = vf_loss / self.gradient_accumulation
                    if i == len(micro_batches) - 1 and self.grad_reducer is not None:
                        self.grad_reducer.begin_sync()
                    loss.backward()
                    if self.grad_reducer is not None:
                        self.grad_reducer.after_backward()
                    met = out.detach()
                    for row in (met if seg or seg_off is not None else [met]):  # one entry per loss micro-batch
                        append_to_dict(dev_metrics, {
                            "critic/vf_loss": row[L.VA_VLOSS_LOSS],
                            "critic/vf_clipfrac": row[L.VA_VLOSS_CLIPFRAC],
                            "critic/vpred_mean": row[L.VA_VLOSS_VPRED_MEAN],
                        })
                grad_norm = self._optimizer_step()
                append_to_dict(dev_metrics, {"critic/grad_norm": grad_norm.detach()})
        self._zero_grad()
        return _to_host(dev_metrics)
