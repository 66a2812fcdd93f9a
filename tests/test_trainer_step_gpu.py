"""RayPPOTrainer / PPOTrainerStep on MI355X: the Ray-free fit() step on real
workers equals the same worker calls issued by hand in the reference's order; a GAE + critic +
adaptive in-reward KL step runs end to end; and a 2-rank (gloo, one GPU) step over a
KK-balanced batch — groups split over ranks, advantages exchanged — equals one process training
on the same reordered batch."""

import copy
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _cfg(est="grpo", kl_in_reward=False, mini_prompts=4):
    from verl_amd.utils.config import AttrDict, actor_config

    return AttrDict(
        algorithm=AttrDict(adv_estimator=est, gamma=1.0, lam=1.0, norm_adv_by_std_in_grpo=True,
                           use_kl_in_reward=kl_in_reward, kl_penalty="low_var_kl",
                           kl_ctrl=AttrDict(type="adaptive", kl_coef=0.01, target_kl=0.001, horizon=100)),
        actor_rollout_ref=AttrDict(
            actor=actor_config(ppo_mini_batch_size=mini_prompts, ppo_micro_batch_size_per_gpu=4,
                               use_kl_loss=not kl_in_reward, kl_loss_coef=0.01, grad_clip=1.0,
                               optim=AttrDict(lr=1e-3, weight_decay=0.01, betas=(0.9, 0.999))),
            rollout=AttrDict(n=4, temperature=1.0, log_prob_micro_batch_size_per_gpu=4)),
        trainer=AttrDict(critic_warmup=0, balance_batch=True))


def _actor_worker(cfg, seed=11):
    from verl_amd.utils.config import AttrDict
    from verl_amd.utils.model import build_qwen2
    from verl_amd.workers.dp_workers import ActorWorker

    c = AttrDict(actor=copy.deepcopy(cfg.actor_rollout_ref.actor), rollout=cfg.actor_rollout_ref.rollout)
    w = ActorWorker(c, rollout_n=cfg.actor_rollout_ref.rollout.n)
    w.init_model(build_qwen2("tiny", device=DEV, seed=seed, attn_implementation="sdpa"))
    w.init_ref_model(build_qwen2("tiny", device=DEV, seed=seed, attn_implementation="sdpa"))
    return w


def _batch(n_prompts=4, seed=3):
    from verl_amd.utils.synthetic import make_grpo_batch

    return make_grpo_batch(n_prompts=n_prompts, n=4, prompt_len=24, response_len=40, vocab=4096, min_prompt=3,
                           dense_responses=False, min_response=5, seed=seed)  # host tensors, as the driver holds


def _params(worker):
    return torch.cat([p.detach().float().reshape(-1) for p in worker.module.parameters()])


def test_fit_step_equals_manual_reference_order():
    from verl_amd.trainer.ppo.core_algos import AdvantageEstimator
    from verl_amd.trainer.ppo.ray_trainer import RayPPOTrainer
    from verl_amd.trainer.ppo.trainer_step import Role

    cfg = _cfg()
    a1, a2 = _actor_worker(cfg), _actor_worker(cfg)
    tr = RayPPOTrainer(cfg, role_worker_mapping={Role.ActorRollout: lambda: a1, Role.RefPolicy: lambda: None})
    met = tr.fit_step(_batch())
    # by hand, the reference's order (ray_trainer.py:1221-1320)
    b = _batch().to(DEV)
    b.batch["response_mask"] = b.batch["attention_mask"][:, -b.batch["responses"].shape[1]:]
    b.batch["old_log_probs"] = a2.compute_log_prob(b).batch["old_log_probs"]
    b.batch["ref_log_prob"] = a2.compute_ref_log_prob(b).batch["ref_log_prob"]
    b.batch["token_level_rewards"] = b.batch["token_level_scores"]
    a2.compute_advantage(b, AdvantageEstimator.GRPO)
    out = a2.update_actor(b)
    assert torch.equal(_params(a1), _params(a2))
    assert met["actor/pg_loss"] == pytest.approx(float(np.mean(out.meta_info["metrics"]["actor/pg_loss"])))
    assert np.isfinite(met["actor/entropy"]) and met["actor/entropy"] > 0


def test_gae_critic_adaptive_kl_step_runs():
    from verl_amd.trainer.ppo.trainer_step import PPOTrainerStep
    from verl_amd.utils.config import critic_config
    from verl_amd.utils.model import build_qwen2_critic
    from verl_amd.workers.dp_workers import CriticWorker

    cfg = _cfg("gae", kl_in_reward=True)
    actor = _actor_worker(cfg)
    ccfg = critic_config(ppo_mini_batch_size=4, rollout_n=4, ppo_micro_batch_size_per_gpu=4, grad_clip=1.0,
                         cliprange_value=0.5)
    critic = CriticWorker(ccfg).init_model(build_qwen2_critic("tiny", device=DEV, seed=5, attn_implementation="sdpa"))
    step = PPOTrainerStep(cfg, actor, critic=critic)
    beta0 = step.kl_ctrl_in_reward.value
    p0 = _params(actor)
    b, met = step.step(_batch(seed=4))
    assert step.kl_ctrl_in_reward.value != beta0
    assert "critic/vf_loss" in met and np.isfinite(met["critic/vf_loss"])
    assert np.isfinite(met["actor/reward_kl_penalty"]) and np.isfinite(met["actor/pg_loss"])
    assert not torch.equal(p0, _params(actor))
    assert torch.isfinite(b.batch["advantages"]).all() and torch.isfinite(b.batch["returns"]).all()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dp_worker(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from verl_amd.trainer.ppo.dp_algos import check_groups_intact
    from verl_amd.trainer.ppo.trainer_step import PPOTrainerStep, shard_batch

    cfg = _cfg(mini_prompts=4)
    actor = _actor_worker(cfg)
    full = _batch(n_prompts=4, seed=8)
    shard = shard_batch(full, balance=True)
    assert not check_groups_intact(shard.non_tensor_batch["uid"])
    PPOTrainerStep(cfg, actor).step(shard)
    if rank == 0:
        torch.save(_params(actor).cpu(), out_path)
        torch.save(full.batch["input_ids"], out_path + ".order")
    dist.destroy_process_group()


def test_dp2_step_with_split_groups_equals_single_process(tmp_path):
    from verl_amd.trainer.ppo.trainer_step import PPOTrainerStep

    out = str(tmp_path / "p.pt")
    mp.spawn(_dp_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    # one process, the same (balanced) row order, the same micro-batch boundaries
    cfg = _cfg(mini_prompts=4)
    actor = _actor_worker(cfg)
    full = _batch(n_prompts=4, seed=8)
    from verl_amd.trainer.ppo.ray_trainer import balance_batch

    balance_batch(full, 2, {})
    assert torch.equal(full.batch["input_ids"], torch.load(out + ".order", weights_only=True))
    PPOTrainerStep(cfg, actor).step(full)
    want = _params(actor).cpu()
    assert torch.allclose(got, want, atol=1e-6, rtol=1e-5), (got - want).abs().max()
