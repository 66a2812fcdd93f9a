"""Ray-free PPO/GRPO training step with the RayPPOTrainer surface (ray_trainer.py:293-400, fit step
ordering :1160-1330), SPMD: every rank runs the same step on its own DP shard of the batch.

The reference's fit() runs on ONE driver process: it holds the whole batch in host memory,
balances it (_balance_batch, :1064-1079), computes advantages there on CPU (:1291-1305), and
ships DP chunks to Ray worker groups for old-logp / ref / values / critic / actor updates. Here
there is no driver and no RPC: each rank (one per MI355X, torch.distributed over RCCL)

  1. receives its shard (``shard_batch``: the DP_COMPUTE_PROTO chunk of the balanced batch,
     decorator.py:375-385) and moves it to the GPU ONCE (``to_device``: the only host->device
     copy of the step; the reference re-pickles the batch for every worker call);
  2. runs the reference's step in the reference's order —
       response_mask -> global_token_num -> reward (reward_fn) -> old_log_prob (+ actor/entropy)
       -> ref_log_prob -> values -> token_level_rewards (in-reward KL) -> advantages
       -> update_critic -> update_actor (after critic_warmup) —
     with the batch-global pieces exchanged over the process group: advantage statistics and
     whitening (dp_algos.compute_advantage_dp), the in-reward KL mean that drives the adaptive
     KL controller (apply_kl_penalty_dp), and the metrics (reduce_metrics over ranks).

``RayPPOTrainer`` in ray_trainer.py keeps the reference constructor on top of this class.
"""

from __future__ import annotations

from enum import Enum
from typing import Callable, Optional

import numpy as np
import torch
import torch.distributed as dist

from ...protocol import DataProto
from ...utils import comm
from . import core_algos
from .core_algos import AdvantageEstimator


class Role(Enum):
    """ray_trainer.py:67-78: the worker roles a trainer maps to resource pools (subclass to add
    roles); here one process per GPU plays the actor (and critic / ref) roles of its DP rank.
    verl_amd.trainer.ppo.ray_trainer re-exports this enum."""

    Actor = 0
    Rollout = 1
    ActorRollout = 2
    Critic = 3
    RefPolicy = 4
    RewardModel = 5
    ActorRolloutRef = 6


_CRITIC_FREE = {
    AdvantageEstimator.GRPO, AdvantageEstimator.GRPO_PASSK, AdvantageEstimator.REINFORCE_PLUS_PLUS,
    AdvantageEstimator.REMAX, AdvantageEstimator.RLOO, AdvantageEstimator.OPO,
    AdvantageEstimator.REINFORCE_PLUS_PLUS_BASELINE, AdvantageEstimator.GPG,
}


def reduce_metrics(metrics: dict) -> dict:
    """utils/metric/utils.py:23-56: mean of each list, max / min for keys naming them."""
    out = {}
    for k, v in metrics.items():
        if "max" in k:
            out[k] = float(np.max(v))
        elif "min" in k:
            out[k] = float(np.min(v))
        else:
            out[k] = float(np.mean(v))
    return out


def _world(group=None) -> int:
    return comm.world(group)


def _rank(group=None) -> int:
    return comm.rank(group)


def reduce_metrics_dp(metrics: dict, group=None) -> dict:
    """Per-rank reduce_metrics, then the mean over ranks (max / min for keys naming them), as the
    reference's collect of DP workers' metric lists followed by reduce_metrics does for equal
    per-rank list lengths. One all-reduce per reduction kind."""
    local = reduce_metrics(metrics)
    if _world(group) == 1 or not local:
        return local
    keys = sorted(local)
    dev = comm.comm_device(group)
    out = {}
    for kind, op in (("max", dist.ReduceOp.MAX), ("min", dist.ReduceOp.MIN), ("mean", dist.ReduceOp.SUM)):
        sel = [k for k in keys if (kind == "max" and "max" in k) or (kind == "min" and "min" in k and "max" not in k)
               or (kind == "mean" and "max" not in k and "min" not in k)]
        if not sel:
            continue
        t = torch.tensor([local[k] for k in sel], dtype=torch.float64, device=dev)
        comm.all_reduce(t, op=op, group=group)
        if kind == "mean":
            t /= _world(group)
        out.update(dict(zip(sel, t.tolist(), strict=True)))
    return out


def shard_batch(batch: DataProto, balance: bool = True, metrics: Optional[dict] = None, group=None) -> DataProto:
    """The DP_COMPUTE_PROTO dispatch of the reference driver on one rank: (optionally) the
    Karmarkar-Karp _balance_batch reorder of the full batch (ray_trainer.py:1204-1205), then this
    rank's equal chunk (decorator.py:375-385). Every rank must call it with the same batch."""
    from .ray_trainer import balance_batch

    w = _world(group)
    if balance and w > 1:
        balance_batch(batch, w, metrics if metrics is not None else {})
    return batch.chunk(w)[_rank(group)] if w > 1 else batch


@torch.no_grad()
def apply_kl_penalty_dp(data: DataProto, kl_ctrl, kl_penalty: str = "kl", group=None):
    """ray_trainer.apply_kl_penalty (ray_trainer.py:153-193) on a DP shard: the kernel computes
    the penalised rewards and each row's masked-mean KL; current_kl is the mean over the rows of
    ALL ranks (one 16-byte all-reduce), so the adaptive controller moves identically everywhere."""
    from ... import kernels as K

    response_mask = data.batch["response_mask"]
    beta = kl_ctrl.value
    rewards, row_kl = K.apply_kl_penalty(data.batch["token_level_scores"], data.batch["old_log_probs"],
                                         data.batch["ref_log_prob"], response_mask, float(beta), kl_penalty)
    t = torch.stack([row_kl.double().sum(), torch.tensor(float(row_kl.numel()), dtype=torch.float64,
                                                          device=row_kl.device)])
    comm.all_reduce(t, group=group)
    batch_size = int(t[1].item())
    current_kl = float((t[0] / t[1]).item())
    kl_ctrl.update(current_kl=current_kl, n_steps=batch_size)
    data.batch["token_level_rewards"] = rewards
    return data, {"actor/reward_kl_penalty": current_kl, "actor/reward_kl_penalty_coeff": beta}


class PPOTrainerStep:
    """One fit() step of RayPPOTrainer (ray_trainer.py:1160-1330) on this rank's shard.

    workers: ``actor`` (ActorWorker: compute_log_prob / compute_advantage / update_actor, and
    compute_ref_log_prob when it also holds the reference policy), optional ``critic``
    (CriticWorker) and ``ref`` (a worker with compute_ref_log_prob). ``reward_fn(batch) ->
    token_level_scores [B, R]`` (or (scores, extra_infos)); when None the batch must carry
    ``token_level_scores`` already (rollout + reward stay outside this path)."""

    def __init__(self, config, actor, critic=None, ref=None, reward_fn: Optional[Callable] = None,
                 process_group=None, device=None):
        self.config = config
        self.actor = actor
        self.critic = critic
        self.ref = ref
        self.reward_fn = reward_fn
        self.group = process_group
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
        self.device = device
        algo = config.algorithm
        self.adv_estimator = AdvantageEstimator(algo.adv_estimator)
        if self.adv_estimator == AdvantageEstimator.GAE:
            self.use_critic = True
        elif self.adv_estimator in _CRITIC_FREE:
            self.use_critic = False
        else:
            raise NotImplementedError
        if self.use_critic and critic is None:
            raise ValueError("GAE needs a critic worker")
        self.use_reference_policy = ref is not None or hasattr(actor, "ref_policy") and actor.ref_policy is not None
        self.kl_ctrl_in_reward = core_algos.get_kl_controller(algo.kl_ctrl) if algo.get("use_kl_in_reward") else None
        # the number of the step about to run: fit() counts from 1 (ray_trainer.py:1099, 1118), so
        # critic_warmup = k holds the actor back for steps 1..k-1
        self.global_steps = 1

    # ------------------------------------------------------------------ host -> device, once
    def to_device(self, batch: DataProto) -> DataProto:
        """The step's single host->device copy (pinned, non-blocking); GPU batches pass through."""
        moved = {}
        for k, v in batch.batch.items():
            if v.device != self.device:
                v = v.pin_memory() if v.device.type == "cpu" and torch.cuda.is_available() else v
                v = v.to(self.device, non_blocking=True)
            moved[k] = v
        for k, v in moved.items():
            batch.batch[k] = v
        return batch

    # ------------------------------------------------------------------ the step
    def step(self, batch: DataProto) -> tuple[DataProto, dict]:
        """ray_trainer.py:1195-1390 from the rollout output on; returns (batch, metrics): the
        workers' reduced metric lists plus the driver's data / timing / throughput metrics
        (metric_utils.py:80-258) over the whole batch of all ranks."""
        from .dp_algos import agg_loss_dp
        from .metric_utils import (SectionTimer, compute_data_metrics, compute_throughout_metrics,
                                   compute_timing_metrics, global_token_num)
        from .ray_trainer import compute_response_mask

        cfg = self.config
        metrics: dict = {}
        timer = SectionTimer(self.device)
        timer.start()
        batch = self.to_device(batch)
        if "response_mask" not in batch.batch.keys():
            batch.batch["response_mask"] = compute_response_mask(batch)
        # the whole batch's per-sequence token counts, as the reference's driver sets them before
        # dispatching DP chunks (ray_trainer.py:1208): MFU and throughput divide by the world size
        batch.meta_info["global_token_num"] = global_token_num(batch.batch["attention_mask"], self.group)

        if self.reward_fn is not None:  # :1209-1218
            with timer.section("reward"):
                res = self.reward_fn(batch)
                scores, extra = res if isinstance(res, tuple) else (res, {})
                batch.batch["token_level_scores"] = scores.to(self.device)
                if extra:
                    batch.non_tensor_batch.update({k: np.array(v) for k, v in extra.items()})

        # old log-probs (+ entropy metric), :1221-1230
        with timer.section("old_log_prob"):
            old = self.actor.compute_log_prob(batch)
            entropys = old.batch["entropys"]
            # over the whole batch as the reference's driver (ray_trainer.py:1224-1228)
            ent = agg_loss_dp(entropys, batch.batch["response_mask"], cfg.actor_rollout_ref.actor.loss_agg_mode,
                              self.group)
            metrics["actor/entropy"] = ent.detach()
            batch.batch["old_log_probs"] = old.batch["old_log_probs"]

        if self.use_reference_policy:  # :1253-1259
            with timer.section("ref"):
                ref_out = (self.ref or self.actor).compute_ref_log_prob(batch)
                batch.batch["ref_log_prob"] = ref_out.batch["ref_log_prob"]

        if self.use_critic:  # :1262-1265
            with timer.section("values"):
                batch.batch["values"] = self.critic.compute_values(batch).batch["values"]

        with timer.section("adv"):
            # rewards (in-reward KL), :1276-1283
            if self.kl_ctrl_in_reward is not None:
                batch, kl_metrics = apply_kl_penalty_dp(batch, self.kl_ctrl_in_reward,
                                                        cfg.algorithm.get("kl_penalty", "kl"), self.group)
                metrics.update(kl_metrics)
            else:
                batch.batch["token_level_rewards"] = batch.batch["token_level_scores"]

            # advantages on the workers (the reference: driver CPU, :1285-1305)
            batch = self.actor.compute_advantage(
                batch, self.adv_estimator, gamma=cfg.algorithm.get("gamma", 1.0), lam=cfg.algorithm.get("lam", 1.0),
                num_repeat=cfg.actor_rollout_ref.rollout.n,
                norm_adv_by_std_in_grpo=cfg.algorithm.get("norm_adv_by_std_in_grpo", True), config=cfg.algorithm)

        # the updates' metrics (dp_actor.DeviceMetrics: an asynchronous device -> host copy) stay unread
        # until both updates are queued, so reading the critic's does not hold back the actor update
        # (ADVICE r5); they are read below, before the step's one metric reduction
        pending = []
        if self.use_critic:  # :1307-1312
            with timer.section("update_critic"):
                critic_out = self.critic.update_critic(batch)
            pending.append(critic_out.meta_info["metrics"])
        if cfg.trainer.get("critic_warmup", 0) <= self.global_steps:  # :1314-1320
            batch.meta_info["multi_turn"] = False
            with timer.section("update_actor"):
                actor_out = self.actor.update_actor(batch)
            pending.append(actor_out.meta_info["metrics"])
        host = {k: [float(v.item())] if isinstance(v, torch.Tensor) else [v] for k, v in metrics.items()}
        for step_metrics in pending:
            host.update({k: (v if isinstance(v, list) else [v]) for k, v in step_metrics.items()})
        timing_raw = timer.read()
        out = reduce_metrics_dp(host, self.group)
        # the driver's metrics after the step (ray_trainer.py:1380-1390)
        out["training/global_step"] = self.global_steps
        out.update(compute_data_metrics(batch, use_critic=self.use_critic, group=self.group))
        out.update(compute_timing_metrics(batch, timing_raw, group=self.group))
        out.update(compute_throughout_metrics(batch, timing_raw, n_gpus=_world(self.group)))
        self.global_steps += 1
        return batch, out
