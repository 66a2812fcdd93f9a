"""Driver-side hot-path functions of verl/trainer/ppo/ray_trainer.py, without Ray.

compute_response_mask (ray_trainer.py:196-211), apply_kl_penalty (:153-193) and
compute_advantage (:214-291) keep their reference signatures and dispatch GAE / GRPO by module
attribute of core_algos, as the reference does (:247, :266), so a replacement of those module
functions is picked up here too. The tensors stay on the device they arrive on: with the
batch already on the MI355X, advantage estimation runs in the gfx950 kernels instead of the
driver CPU.
"""

from __future__ import annotations

from typing import Optional

import torch

from ... import kernels as K
from ...protocol import DataProto
from . import core_algos
from .core_algos import AdvantageEstimator
from .trainer_step import Role  # ray_trainer.py:67-78; one enum for the mapping keys and the step


def apply_kl_penalty(data: DataProto, kl_ctrl, kl_penalty="kl"):
    """ray_trainer.py:153-193: token_level_rewards = scores - beta * kl * mask; adaptive beta update."""
    response_mask = data.batch["response_mask"]
    scores = data.batch["token_level_scores"]
    batch_size = data.batch.batch_size[0]
    beta = kl_ctrl.value
    rewards, row_kl = K.apply_kl_penalty(
        scores, data.batch["old_log_probs"], data.batch["ref_log_prob"], response_mask, float(beta), kl_penalty
    )
    current_kl = torch.mean(row_kl, dim=0).item()
    kl_ctrl.update(current_kl=current_kl, n_steps=batch_size)
    data.batch["token_level_rewards"] = rewards
    return data, {"actor/reward_kl_penalty": current_kl, "actor/reward_kl_penalty_coeff": beta}


def compute_response_mask(data: DataProto):
    """ray_trainer.py:196-211."""
    R = data.batch["responses"].size(1)
    return data.batch["attention_mask"][:, -R:]


def compute_advantage(
    data: DataProto,
    adv_estimator: AdvantageEstimator,
    gamma: float = 1.0,
    lam: float = 1.0,
    num_repeat: int = 1,
    norm_adv_by_std_in_grpo: bool = True,
    config: Optional[dict] = None,
) -> DataProto:
    """ray_trainer.py:214-291."""
    if "response_mask" not in data.batch.keys():
        data.batch["response_mask"] = compute_response_mask(data)
    if adv_estimator == AdvantageEstimator.GAE:
        adv, ret = core_algos.compute_gae_advantage_return(
            token_level_rewards=data.batch["token_level_rewards"],
            values=data.batch["values"],
            response_mask=data.batch["response_mask"],
            gamma=gamma,
            lam=lam,
        )
        data.batch["advantages"] = adv
        data.batch["returns"] = ret
        if config is not None and config.get("use_pf_ppo", False):
            data = core_algos.compute_pf_ppo_reweight_data(
                data, config.pf_ppo.reweight_method, config.pf_ppo.weight_pow
            )
    elif adv_estimator == AdvantageEstimator.GRPO:
        adv, ret = core_algos.compute_grpo_outcome_advantage(
            token_level_rewards=data.batch["token_level_rewards"],
            response_mask=data.batch["response_mask"],
            index=data.non_tensor_batch["uid"],
            norm_adv_by_std_in_grpo=norm_adv_by_std_in_grpo,
        )
        data.batch["advantages"] = adv
        data.batch["returns"] = ret
    else:
        fn = core_algos.get_adv_estimator_fn(adv_estimator)
        kwargs = {
            "token_level_rewards": data.batch["token_level_rewards"],
            "response_mask": data.batch["response_mask"],
            "config": config,
        }
        if "uid" in data.non_tensor_batch:
            kwargs["index"] = data.non_tensor_batch["uid"]
        if "reward_baselines" in data.batch:
            kwargs["reward_baselines"] = data.batch["reward_baselines"]
        adv, ret = fn(**kwargs)
        data.batch["advantages"] = adv
        data.batch["returns"] = ret
    return data


def balance_batch(batch: DataProto, world_size: int, metrics: dict, logging_prefix: str = "global_seqlen"):
    """RayPPOTrainer._balance_batch (ray_trainer.py:1064-1079) without Ray: reorder ``batch`` in
    place so the equal ``chunk(world_size)`` of DP_COMPUTE_PROTO gives every rank a similar total
    token count (Karmarkar-Karp, equal partition sizes); balance statistics go into ``metrics``."""
    from ...utils.seqlen_balancing import get_seqlen_balanced_partitions, log_seqlen_unbalance

    am = batch.batch["attention_mask"]
    seqlens = am.view(am.shape[0], -1).sum(-1).tolist()
    parts = get_seqlen_balanced_partitions(seqlens, k_partitions=world_size, equal_size=True)
    batch.reorder(torch.tensor([j for p in parts for j in p]))
    metrics.update(log_seqlen_unbalance(seqlen_list=seqlens, partitions=parts, prefix=logging_prefix))


def filter_groups(batch: DataProto, metric: str = "acc"):
    """DAPO dynamic sampling filter (recipe/dapo/dapo_ray_trainer.py:199-237): keep the responses
    of every prompt (uid) whose ``metric`` has a non-zero population std across its responses,
    plus singleton groups. ``metric`` is a non-tensor key, or "seq_final_reward" /
    "seq_reward" (row sums of token_level_rewards / token_level_scores, computed here as the
    reference does). Returns (kept batch, number of kept prompts)."""
    import numpy as np

    if metric == "seq_final_reward":
        batch.non_tensor_batch["seq_final_reward"] = batch.batch["token_level_rewards"].sum(dim=-1).cpu().numpy()
    elif metric == "seq_reward":
        batch.non_tensor_batch["seq_reward"] = batch.batch["token_level_scores"].sum(dim=-1).cpu().numpy()
    uids = batch.non_tensor_batch["uid"]
    vals: dict = {}
    for uid, v in zip(uids, batch.non_tensor_batch[metric], strict=True):
        vals.setdefault(uid, []).append(v)
    kept = {uid for uid, vs in vals.items() if np.std(vs) > 0 or len(vs) == 1}
    idx = [i for i, uid in enumerate(uids) if uid in kept]
    return batch[idx], len(kept)


class ResourcePoolManager:
    """ray_trainer.py:81-126 without Ray: the GPUs are the torch.distributed ranks of this job, so
    the spec is recorded for reference and the pools are this process group."""

    def __init__(self, resource_pool_spec: Optional[dict] = None, mapping: Optional[dict] = None):
        self.resource_pool_spec = resource_pool_spec or {}
        self.mapping = mapping or {}

    def create_resource_pool(self):
        return None

    def get_n_gpus(self) -> int:
        import torch.distributed as dist

        return dist.get_world_size() if dist.is_initialized() else 1


class RayPPOTrainer:
    """The reference's trainer surface (ray_trainer.py:293-400 constructor, :823 init_workers,
    :1081 fit) for an SPMD job: every rank constructs it with the same arguments.

    role_worker_mapping maps a Role to a zero-argument factory returning this rank's worker
    (ActorWorker / CriticWorker; Role.RefPolicy may map to the actor itself when it holds the
    reference policy). Rollout generation and reward models are outside this path: ``fit`` takes
    rollout batches (input_ids / attention_mask / position_ids / responses [+ uid, scores]), and
    reward_fn(batch) -> token_level_scores supplies the reward when the batch has none."""

    def __init__(self, config, tokenizer=None, role_worker_mapping: Optional[dict] = None, resource_pool_manager=None,
                 ray_worker_group_cls=None, processor=None, reward_fn=None, val_reward_fn=None, train_dataset=None,
                 val_dataset=None, collate_fn=None, train_sampler=None, device_name="cuda"):

        self.config = config
        self.tokenizer = tokenizer
        self.processor = processor
        self.reward_fn = reward_fn
        self.val_reward_fn = val_reward_fn
        self.role_worker_mapping = role_worker_mapping or {}
        self.resource_pool_manager = resource_pool_manager or ResourcePoolManager()
        self.device_name = device_name
        assert Role.ActorRollout in self.role_worker_mapping, f"{self.role_worker_mapping.keys()=}"
        self.use_reference_policy = Role.RefPolicy in self.role_worker_mapping
        self.use_rm = Role.RewardModel in self.role_worker_mapping
        self.use_critic = AdvantageEstimator(config.algorithm.adv_estimator) == AdvantageEstimator.GAE
        self.step_runner = None
        self.global_steps = 0

    def init_workers(self):
        """ray_trainer.py:823-907: build the role workers (here: call the factories)."""
        from .trainer_step import PPOTrainerStep

        self.actor_rollout_wg = self.role_worker_mapping[Role.ActorRollout]()
        self.critic_wg = self.role_worker_mapping[Role.Critic]() if self.use_critic else None
        ref = None
        if self.use_reference_policy:
            ref = self.role_worker_mapping[Role.RefPolicy]()
            if ref is None:
                ref = self.actor_rollout_wg
        self.ref_policy_wg = ref
        self.step_runner = PPOTrainerStep(self.config, self.actor_rollout_wg, critic=self.critic_wg, ref=ref,
                                          reward_fn=self.reward_fn)

    def fit_step(self, batch: DataProto) -> dict:
        """One iteration of fit() (ray_trainer.py:1195-1330) on this rank's shard. Steps are
        numbered from 1 as in fit() (global_steps = 0, then += 1 before the first step,
        ray_trainer.py:1099, 1118), which is what critic_warmup compares against (:1315)."""
        if self.step_runner is None:
            self.init_workers()
        if self.global_steps == 0:
            self.global_steps = 1
        self.step_runner.global_steps = self.global_steps
        _, metrics = self.step_runner.step(batch)
        metrics["training/global_step"] = self.global_steps
        self.global_steps += 1
        return metrics

    def fit(self, batches) -> list[dict]:
        """ray_trainer.py:1081-1411 over an iterable of rollout shards; returns the per-step metrics."""
        self.global_steps = 0
        return [self.fit_step(b) for b in batches]
