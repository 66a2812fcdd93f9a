"""Attribute-style config dicts (the reference passes omegaconf DictConfig objects; the hot path
only needs ``cfg.key`` and ``cfg.get(key, default)``)."""

from __future__ import annotations

from typing import Any


class AttrDict(dict):
    """dict with attribute access; nested dicts are wrapped on read."""

    def __getattr__(self, name: str) -> Any:
        try:
            v = self[name]
        except KeyError as e:
            raise AttributeError(name) from e
        if isinstance(v, dict) and not isinstance(v, AttrDict):
            v = AttrDict(v)
            self[name] = v
        return v

    def __setattr__(self, name: str, value: Any) -> None:
        self[name] = value

    def get(self, key, default=None):
        v = super().get(key, default)
        if isinstance(v, dict) and not isinstance(v, AttrDict):
            v = AttrDict(v)
        return v


def actor_config(**overrides) -> AttrDict:
    """Defaults of verl/trainer/config/actor/actor.yaml:9-111 + dp_actor.yaml:17-73 that the
    actor-update path reads."""
    cfg = AttrDict(
        strategy="fsdp",
        ppo_mini_batch_size=256,
        ppo_micro_batch_size=None,
        ppo_micro_batch_size_per_gpu=None,
        use_dynamic_bsz=False,
        ppo_max_token_len_per_gpu=16384,
        clip_ratio=0.2,
        clip_ratio_low=0.2,
        clip_ratio_high=0.2,
        policy_loss=AttrDict(loss_mode="vanilla", clip_cov_ratio=0.0002, clip_cov_lb=1.0, clip_cov_ub=5.0,
                             kl_cov_ratio=0.0002, ppo_kl_coef=0.1),
        clip_ratio_c=3.0,
        loss_agg_mode="token-mean",
        entropy_coeff=0,
        use_kl_loss=False,
        use_torch_compile=True,
        kl_loss_coef=0.001,
        kl_loss_type="low_var_kl",
        ppo_epochs=1,
        shuffle=False,
        grad_clip=1.0,
        ulysses_sequence_parallel_size=1,
        entropy_from_logits_with_chunking=False,
        entropy_checkpointing=False,
        use_remove_padding=True,
        use_fused_kernels=False,
        fused_logprob_no_grad=False,
        fused_mlp_no_grad=False,
        fused_mlp_train=False,
        fused_qkv=False,
        # (verl_amd) responses per update forward/backward pass; None = ppo_micro_batch_size_per_gpu
        compute_micro_batch_size_per_gpu=None,
        # (verl_amd) use_dynamic_bsz: tokens per update pass holding several token-budget micro-batches
        compute_max_token_len_per_gpu=None,
        optim=AttrDict(lr=1e-6, weight_decay=0.01, betas=(0.9, 0.999), lr_warmup_steps=-1, lr_warmup_steps_ratio=0.0,
                       min_lr_ratio=0.0, num_cycles=0.5, warmup_style="constant", total_training_steps=-1),
    )
    for k, v in overrides.items():
        cfg[k] = v
    return cfg


def critic_config(**overrides) -> AttrDict:
    """Defaults of verl/trainer/config/critic/critic.yaml + dp_critic.yaml that the critic-update
    path reads (mini-batch sizes are inherited from the actor there; set them explicitly here)."""
    cfg = AttrDict(
        strategy="fsdp",
        rollout_n=1,
        ppo_mini_batch_size=256,
        ppo_micro_batch_size=None,
        ppo_micro_batch_size_per_gpu=None,
        forward_micro_batch_size=None,
        forward_micro_batch_size_per_gpu=None,
        use_dynamic_bsz=False,
        ppo_max_token_len_per_gpu=32768,
        forward_max_token_len_per_gpu=32768,
        ppo_epochs=1,
        shuffle=False,
        cliprange_value=0.5,
        loss_agg_mode="token-mean",
        grad_clip=1.0,
        ulysses_sequence_parallel_size=1,
        # (verl_amd) responses per update forward/backward pass; None = ppo_micro_batch_size_per_gpu
        compute_micro_batch_size_per_gpu=None,
        # (verl_amd) use_dynamic_bsz: tokens per update pass holding several token-budget micro-batches
        compute_max_token_len_per_gpu=None,
        model=AttrDict(use_remove_padding=False, enable_gradient_checkpointing=True),
        optim=AttrDict(lr=1e-5, weight_decay=0.01, betas=(0.9, 0.999), lr_warmup_steps_ratio=0.0, min_lr_ratio=None,
                       warmup_style="constant", total_training_steps=-1),
    )
    for k, v in overrides.items():
        cfg[k] = v
    return cfg
