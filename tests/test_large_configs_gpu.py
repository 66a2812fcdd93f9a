"""BASELINE configs 3 and 5 at their real model sizes on ONE MI355X (their 8-GPU runs are the
driver's; no checkpoints exist here, so random init of the public architectures):

* config 5, DAPO on Qwen2.5-7B (recipe/dapo): dynamic sampling (filter_groups on the sequence
  reward, dapo_ray_trainer.py:199-237), token-level loss (loss_agg_mode "token-mean"),
  decoupled clip (clip_ratio_low 0.2 / clip_ratio_high 0.28), no KL loss and no reference
  policy; one Ray-free fit step (PPOTrainerStep) with the sharded optimizer manager;
* config 3's critic, Llama-3-8B as LlamaForTokenClassification (fsdp_workers.py:1018-1031):
  values -> GAE advantages / returns (the fused scan + whitening kernels) -> one critic update.

Property checks (no reference outputs exist for these sizes): finite losses / gradient norms,
weights move, the filter keeps exactly the groups with a non-zero reward std, advantages are zero
off the response mask, and GAE advantages come out whitened over the mask (mean 0, std 1)."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _fresh_device_memory():
    """Each test holds a 7-8B model's state (~150-180 GB): release the previous test's before."""
    import gc

    gc.collect()
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats()
    yield
    gc.collect()
    torch.cuda.empty_cache()


def _qwen25_7b():
    from verl_amd.utils.model import build_qwen2

    model = build_qwen2("7b", device=DEV, seed=0, attn_implementation="sdpa")
    n = sum(p.numel() for p in model.parameters())
    assert 7.5e9 < n < 7.7e9, n
    return model


def test_dapo_qwen25_7b_dynamic_sampling_token_mean_one_step():
    from verl_amd.trainer.ppo.ray_trainer import filter_groups
    from verl_amd.trainer.ppo.trainer_step import PPOTrainerStep
    from verl_amd.utils.config import AttrDict, actor_config
    from verl_amd.utils.synthetic import make_grpo_batch
    from verl_amd.workers.dp_workers import ActorWorker

    n = 4
    cfg = AttrDict(
        algorithm=AttrDict(adv_estimator="grpo", gamma=1.0, lam=1.0, norm_adv_by_std_in_grpo=True,
                           use_kl_in_reward=False),
        actor_rollout_ref=AttrDict(
            actor=actor_config(ppo_mini_batch_size=8, ppo_micro_batch_size_per_gpu=4, use_kl_loss=False,
                               clip_ratio_low=0.2, clip_ratio_high=0.28, clip_ratio_c=10.0,
                               loss_agg_mode="token-mean", grad_clip=1.0,
                               optim=AttrDict(lr=1e-6, weight_decay=0.1, betas=(0.9, 0.999))),
            rollout=AttrDict(n=n, temperature=1.0, log_prob_micro_batch_size_per_gpu=4)),
        trainer=AttrDict(critic_warmup=0, balance_batch=False))
    batch = make_grpo_batch(n_prompts=6, n=n, prompt_len=64, response_len=256, vocab=152064, min_prompt=16,
                            dense_responses=False, min_response=32, seed=5)
    # DAPO dynamic sampling: one Bernoulli score per response; make two groups uniform so they drop
    scores = batch.batch["token_level_scores"]
    uids = batch.non_tensor_batch["uid"]
    groups = list(dict.fromkeys(uids.tolist()))
    rows0 = [i for i, u in enumerate(uids) if u == groups[0]]
    rows1 = [i for i, u in enumerate(uids) if u == groups[1]]
    resp_len = batch.batch["attention_mask"][:, -scores.shape[1]:].sum(-1)
    for r, val in [(i, 1.0) for i in rows0] + [(i, 0.0) for i in rows1]:
        scores[r].zero_()
        scores[r, int(resp_len[r]) - 1] = val
    batch.batch["token_level_rewards"] = scores.clone()
    seq = scores.sum(-1).numpy()
    want = {u for u in groups if np.std([seq[i] for i, x in enumerate(uids) if x == u]) > 0}
    kept, n_kept = filter_groups(batch, "seq_final_reward")
    assert n_kept == len(want) and set(kept.non_tensor_batch["uid"].tolist()) == want
    assert groups[0] not in want and groups[1] not in want
    kept = kept[: (len(kept) // 8) * 8]  # whole mini-batches (the recipe refills to train_batch_size)
    assert len(kept) >= 8
    cfg.actor_rollout_ref.actor.ppo_mini_batch_size = len(kept) // n

    worker = ActorWorker(AttrDict(actor=cfg.actor_rollout_ref.actor, rollout=cfg.actor_rollout_ref.rollout),
                         rollout_n=n)
    worker.init_model(_qwen25_7b(), bucket_mb=1024, zero=True)
    before = [p.detach().clone() for p in list(worker.module.parameters())[:3]]
    step = PPOTrainerStep(cfg, worker)
    out, met = step.step(kept)
    for k in ("actor/pg_loss", "actor/grad_norm", "actor/pg_clipfrac", "actor/entropy"):
        assert np.isfinite(met[k]), (k, met[k])
    assert met["actor/grad_norm"] > 0
    assert "actor/kl_loss" not in met  # use_kl_loss False: no reference policy, no KL term
    adv = out.batch["advantages"]
    m = out.batch["response_mask"].bool()
    assert torch.isfinite(adv).all() and (adv[~m] == 0).all()
    after = list(worker.module.parameters())[:3]
    assert any(not torch.equal(a, b) for a, b in zip(after, before, strict=True))
    print("dapo 7b", {k: round(v, 5) for k, v in met.items() if k.startswith("actor/")},
          "peak GB", torch.cuda.max_memory_allocated() / 1e9)


def test_llama3_8b_critic_gae_values_and_update():
    from verl_amd.trainer.ppo import ray_trainer
    from verl_amd.trainer.ppo.core_algos import AdvantageEstimator
    from verl_amd.utils.config import critic_config
    from verl_amd.utils.model import build_llama_critic
    from verl_amd.utils.synthetic import make_grpo_batch
    from verl_amd.workers.dp_workers import CriticWorker

    model = build_llama_critic("8b", device=DEV, seed=1, attn_implementation="sdpa")
    assert 7.4e9 < sum(p.numel() for p in model.parameters()) < 7.6e9  # no lm_head: a 1-wide score head
    ccfg = critic_config(ppo_mini_batch_size=2, rollout_n=4, ppo_micro_batch_size_per_gpu=2, grad_clip=1.0,
                         cliprange_value=0.5, forward_micro_batch_size_per_gpu=4)
    critic = CriticWorker(ccfg).init_model(model, bucket_mb=1024, zero=True)
    data = make_grpo_batch(n_prompts=2, n=4, prompt_len=64, response_len=256, vocab=128256, min_prompt=16,
                           dense_responses=False, min_response=32, seed=9, device=DEV)
    data.meta_info.update(temperature=1.0, micro_batch_size=4, use_dynamic_bsz=False)
    b = data.batch
    b["response_mask"] = b["attention_mask"][:, -b["responses"].shape[1]:]
    b["values"] = critic.compute_values(data).batch["values"]
    m = b["response_mask"].bool()
    assert torch.isfinite(b["values"]).all() and (b["values"][~m] == 0).all()
    b["token_level_rewards"] = b["token_level_scores"]
    ray_trainer.compute_advantage(data, AdvantageEstimator.GAE, gamma=1.0, lam=0.95)
    adv, ret = b["advantages"], b["returns"]
    assert torch.isfinite(adv).all() and torch.isfinite(ret).all()
    am = adv[m].double()
    assert abs(float(am.mean())) < 1e-4 and abs(float(am.std()) - 1.0) < 1e-3  # whitened over the mask
    before = [p.detach().clone() for p in list(model.parameters())[-2:]]
    out = critic.update_critic(data)
    met = out.meta_info["metrics"]
    assert np.isfinite(np.mean(met["critic/vf_loss"])) and np.mean(met["critic/grad_norm"]) > 0
    assert any(not torch.equal(a, b_) for a, b_ in zip(list(model.parameters())[-2:], before, strict=True))
    print("llama 8b critic", {k: float(np.mean(v)) for k, v in met.items()},
          "peak GB", torch.cuda.max_memory_allocated() / 1e9)
