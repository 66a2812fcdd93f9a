"""ORACLE — CPU restatement of the rfahrn/verl actor-update hot path (TEST INFRASTRUCTURE).

This module is the checker, never the product: only ``tests/``, ``__graft_entry__.smoke()``
and the ``cpu_baseline`` leg of ``bench.py`` may import it. It restates, in eager PyTorch on
the CPU, the reference functions listed in SURVEY.md §8(a), keeping the reference's op order,
clamps, epsilons, dtype promotions and error surface so that its fp32 results are what the
reference computes on the same inputs (and its float64 twin, obtained by passing float64
tensors, is the error-budget reference).

Pinning: importing the reference itself was denied in this environment, so
the restatement is pinned by the reference's own known-answer tests and properties
(tests/utils/test_torch_functional.py:55-66 masked_mean KATs; tests/trainer/ppo/
test_core_algos_on_cpu.py:134-188 GAE multi-turn property; the registry error texts of
test_core_algos_on_cpu.py:119-131; the hand-derivable GRPO input of
tests/trainer/config/test_algo_config_on_cpu.py:190-192) plus hand-derived KATs from the
source semantics. See tests/test_oracle_kats.py.

Every function cites the reference file:line it restates (paths relative to verl/).
"""

from __future__ import annotations

from collections import OrderedDict

import numpy as np
import torch
import torch.nn.functional as F

# ----------------------------------------------------------------------------- masked stats


def masked_sum(values, mask, axis=None):
    """utils/torch_functional.py:163-168 — zero NaNs outside the mask, then sum(values*mask)."""
    kept = torch.where(mask.bool(), values, 0.0)
    return (kept * mask).sum(axis=axis)


def masked_mean(values, mask, axis=None):
    """utils/torch_functional.py:171-185 — masked_sum / (mask.sum + 1e-8)."""
    return masked_sum(values, mask, axis) / (mask.sum(axis=axis) + 1e-8)


def masked_var(values, mask, unbiased=True):
    """utils/torch_functional.py:188-203 — masked variance; Bessel factor n/(n-1)."""
    centred = values - masked_mean(values, mask)
    var = masked_mean(centred**2, mask)
    if unbiased:
        n = mask.sum()
        if n == 0:
            raise ValueError("At least one element in the mask has to be 1.")
        if n == 1:
            raise ValueError("The sum of the mask is one, which can cause a division by zero.")
        var = var * (n / (n - 1))
    return var


def masked_whiten(values, mask, shift_mean=True):
    """utils/torch_functional.py:206-223."""
    mu = masked_mean(values, mask)
    var = masked_var(values, mask)
    out = (values - mu) * torch.rsqrt(var + 1e-8)
    if not shift_mean:
        out += mu
    return out


# ----------------------------------------------------------------------------- log-prob / entropy


def apply_temperature(logits, temperature):
    """workers/actor/dp_actor.py:182 — logits.div_(temperature), in the logits' own dtype."""
    return logits.clone().div_(temperature)


def logprobs_from_logits(logits, labels):
    """utils/torch_functional.py:116-133 (logprobs_from_logits_v2, the CPU path).

    fp32/fp64: gather - per-row logsumexp; bf16/fp16: per-row log_softmax then gather.
    """
    if logits.dtype in (torch.float32, torch.float64):
        picked = torch.gather(logits, dim=-1, index=labels.unsqueeze(-1)).squeeze(-1)
        lse = torch.stack([torch.logsumexp(row, dim=-1) for row in logits])
        return picked - lse
    rows = []
    for row, lab in zip(logits, labels, strict=True):
        rows.append(F.log_softmax(row, dim=-1).gather(dim=-1, index=lab.unsqueeze(-1)).squeeze(-1))
    return torch.stack(rows)


def logprobs_fp32_math(logits, labels):
    """flash-attn cross_entropy_loss semantics (torch_functional.py:95-100): the loss is computed in
    fp32 from the (possibly bf16) logits: logp = x[label] - logsumexp(x) with fp32 upcast."""
    x = logits.float()
    return logprobs_from_logits(x, labels)


def entropy_from_logits(logits):
    """utils/torch_functional.py:145-149."""
    p = torch.nn.functional.softmax(logits, dim=-1)
    return torch.logsumexp(logits, dim=-1) - torch.sum(p * logits, dim=-1)


# ----------------------------------------------------------------------------- losses


def agg_loss(loss_mat, loss_mask, loss_agg_mode):
    """trainer/ppo/core_algos.py:686-719."""
    if loss_agg_mode == "token-mean":
        return masked_mean(loss_mat, loss_mask)
    if loss_agg_mode == "seq-mean-token-sum":
        return torch.mean(torch.sum(loss_mat * loss_mask, dim=-1))
    if loss_agg_mode == "seq-mean-token-mean":
        per_seq = torch.sum(loss_mat * loss_mask, dim=-1) / torch.sum(loss_mask, dim=-1)
        return torch.mean(per_seq)
    if loss_agg_mode == "seq-mean-token-sum-norm":
        return torch.sum(torch.sum(loss_mat * loss_mask, dim=-1)) / loss_mask.shape[-1]
    raise ValueError(f"Invalid loss_agg_mode: {loss_agg_mode}")


def compute_policy_loss(
    old_log_prob,
    log_prob,
    advantages,
    response_mask,
    cliprange=None,
    cliprange_low=None,
    cliprange_high=None,
    clip_ratio_c=3.0,
    loss_agg_mode="token-mean",
):
    """trainer/ppo/core_algos.py:722-794 — dual-clip PPO; returns (pg_loss, clipfrac, ppo_kl,
    clipfrac_lower)."""
    assert clip_ratio_c > 1.0, (
        "The lower bound of the clip_ratio_c for dual-clip PPO should be greater than 1.0,"
        + f" but get the value: {clip_ratio_c}."
    )
    lo = cliprange if cliprange_low is None else cliprange_low
    hi = cliprange if cliprange_high is None else cliprange_high
    neg_kl = torch.clamp(log_prob - old_log_prob, min=-20.0, max=20.0)
    ratio = torch.exp(neg_kl)
    ppo_kl = masked_mean(-neg_kl, response_mask)
    loss_unclipped = -advantages * ratio
    loss_clipped = -advantages * torch.clamp(ratio, 1 - lo, 1 + hi)
    loss_max = torch.maximum(loss_unclipped, loss_clipped)
    clipfrac = masked_mean(torch.gt(loss_clipped, loss_unclipped).float(), response_mask)
    loss_dual = -advantages * clip_ratio_c
    loss_dual_min = torch.min(loss_dual, loss_max)
    clipfrac_lower = masked_mean(torch.gt(loss_max, loss_dual) * (advantages < 0).float(), response_mask)
    per_token = torch.where(advantages < 0, loss_dual_min, loss_max)
    pg_loss = agg_loss(per_token, response_mask, loss_agg_mode)
    return pg_loss, clipfrac, ppo_kl, clipfrac_lower


def clip_by_value(x, tensor_min, tensor_max):
    """utils/torch_functional.py:136-142."""
    return torch.max(torch.min(x, tensor_max), tensor_min)


def compute_value_loss(vpreds, returns, values, response_mask, cliprange_value, loss_agg_mode="token-mean"):
    """trainer/ppo/core_algos.py:992-1031 — clipped value loss and clip fraction."""
    vpredclipped = clip_by_value(vpreds, values - cliprange_value, values + cliprange_value)
    vf_losses1 = (vpreds - returns) ** 2
    vf_losses2 = (vpredclipped - returns) ** 2
    clipped_vf_losses = torch.max(vf_losses1, vf_losses2)
    vf_loss = 0.5 * agg_loss(clipped_vf_losses, response_mask, loss_agg_mode)
    vf_clipfrac = masked_mean(torch.gt(vf_losses2, vf_losses1).float(), response_mask)
    return vf_loss, vf_clipfrac


def kl_penalty(logprob, ref_logprob, kl_penalty):
    """trainer/ppo/core_algos.py:1034-1069."""
    if kl_penalty in ("kl", "k1"):
        return logprob - ref_logprob
    if kl_penalty == "abs":
        return (logprob - ref_logprob).abs()
    if kl_penalty in ("mse", "k2"):
        return 0.5 * (logprob - ref_logprob).square()
    if kl_penalty in ("low_var_kl", "k3"):
        k = torch.clamp(ref_logprob - logprob, min=-20, max=20)
        return torch.clamp((torch.exp(k) - k - 1).contiguous(), min=-10, max=10)
    raise NotImplementedError


def actor_loss(
    old_log_prob,
    log_prob,
    advantages,
    response_mask,
    clip_ratio=0.2,
    clip_ratio_low=None,
    clip_ratio_high=None,
    clip_ratio_c=3.0,
    loss_agg_mode="token-mean",
    entropy=None,
    entropy_coeff=0.0,
    ref_log_prob=None,
    kl_loss_type="low_var_kl",
    kl_loss_coef=0.001,
    grad_scale=1.0,
):
    """workers/actor/dp_actor.py:400-469 — the per-micro-batch loss the actor back-propagates:
    (pg_loss - coeff*agg(entropy) + kl_coef*agg(kl_penalty)) * grad_scale, and the metrics."""
    pg_loss, clipfrac, ppo_kl, clipfrac_lower = compute_policy_loss(
        old_log_prob,
        log_prob,
        advantages,
        response_mask,
        cliprange=clip_ratio,
        cliprange_low=clip_ratio_low if clip_ratio_low is not None else clip_ratio,
        cliprange_high=clip_ratio_high if clip_ratio_high is not None else clip_ratio,
        clip_ratio_c=clip_ratio_c,
        loss_agg_mode=loss_agg_mode,
    )
    policy_loss = pg_loss
    ent_loss = None
    if entropy_coeff != 0:
        ent_loss = agg_loss(entropy, response_mask, loss_agg_mode)
        policy_loss = pg_loss - ent_loss * entropy_coeff
    kl_loss = None
    if ref_log_prob is not None:
        kl_loss = agg_loss(kl_penalty(log_prob, ref_log_prob, kl_loss_type), response_mask, loss_agg_mode)
        policy_loss = policy_loss + kl_loss * kl_loss_coef
    loss = policy_loss * grad_scale
    return loss, dict(
        pg_loss=pg_loss, pg_clipfrac=clipfrac, ppo_kl=ppo_kl, pg_clipfrac_lower=clipfrac_lower,
        kl_loss=kl_loss, entropy_loss=ent_loss,
    )


# ----------------------------------------------------------------------------- advantages


def _groups(index):
    """Rows of each uid, in first-appearance order of the uid and row order inside a group
    (core_algos.py:290-291 appends in row order)."""
    groups = OrderedDict()
    for i in range(len(index)):
        groups.setdefault(index[i], []).append(i)
    return groups


def compute_grpo_outcome_advantage(token_level_rewards, response_mask, index, epsilon=1e-6,
                                   norm_adv_by_std_in_grpo=True):
    """trainer/ppo/core_algos.py:246-308 — note the UNMASKED row sum (:282), unbiased std, and
    (mean, std) = (0, 1) for singleton groups (:293-295)."""
    scores = token_level_rewards.sum(dim=-1)
    with torch.no_grad():
        stats = {}
        for uid, rows in _groups(index).items():
            members = [scores[i] for i in rows]
            if len(members) == 1:
                stats[uid] = (torch.tensor(0.0), torch.tensor(1.0))
            else:
                stats[uid] = (torch.mean(torch.tensor(members)), torch.std(torch.tensor([members])))
        for i in range(scores.shape[0]):
            mean, std = stats[index[i]]
            if norm_adv_by_std_in_grpo:
                scores[i] = (scores[i] - mean) / (std + epsilon)
            else:
                scores[i] = scores[i] - mean
        scores = scores.unsqueeze(-1) * response_mask
    return scores, scores


def compute_rloo_outcome_advantage(token_level_rewards, response_mask, index, epsilon=1e-6):
    """trainer/ppo/core_algos.py:428-476."""
    scores = token_level_rewards.sum(dim=-1)
    with torch.no_grad():
        groups = _groups(index)
        means = {}
        for uid, rows in groups.items():
            members = [scores[i] for i in rows]
            means[uid] = torch.tensor(0.0) if len(members) == 1 else torch.mean(torch.tensor(members))
        for i in range(scores.shape[0]):
            n = len(groups[index[i]])
            if n > 1:
                scores[i] = scores[i] * n / (n - 1) - means[index[i]] * n / (n - 1)
        scores = scores.unsqueeze(-1) * response_mask
    return scores, scores


def compute_reinforce_plus_plus_baseline_outcome_advantage(token_level_rewards, response_mask, index,
                                                           epsilon=1e-6):
    """trainer/ppo/core_algos.py:376-424."""
    R = token_level_rewards.shape[-1]
    scores = token_level_rewards.sum(dim=-1)
    with torch.no_grad():
        means = {}
        for uid, rows in _groups(index).items():
            members = [scores[i] for i in rows]
            means[uid] = torch.tensor(0.0) if len(members) == 1 else torch.mean(torch.tensor(members))
        for i in range(scores.shape[0]):
            scores[i] = scores[i] - means[index[i]]
        scores = scores.unsqueeze(-1).tile([1, R]) * response_mask
        scores = masked_whiten(scores, response_mask) * response_mask
    return scores, scores


def compute_grpo_passk_outcome_advantage(token_level_rewards, response_mask, index, epsilon=1e-6, norm=True):
    """trainer/ppo/core_algos.py:311-370 — the group's best response gets r_max - r_second_max."""
    scores = token_level_rewards.sum(dim=-1)
    adv = torch.zeros_like(scores)
    with torch.no_grad():
        for uid, rows in _groups(index).items():
            rewards = torch.stack([scores[i] for i in rows])
            if rewards.numel() < 2:
                raise ValueError(f"Pass@k requires at least 2 samples per group. Got {rewards.numel()} for group {uid}.")
            top, top_idx = torch.topk(rewards, 2)
            a = top[0] - top[1]
            if norm:
                a = a / (torch.std(rewards) + epsilon)
            adv[rows[top_idx[0].item()]] = a
    adv = adv.unsqueeze(-1) * response_mask
    return adv, adv


def compute_opo_outcome_advantage(token_level_rewards, response_mask, index, epsilon=1e-6):
    """trainer/ppo/core_algos.py:479-530 — length-weighted baseline, 0 for singleton groups."""
    lengths = response_mask.sum(dim=-1)
    scores = token_level_rewards.sum(dim=-1)
    with torch.no_grad():
        base = {}
        for uid, rows in _groups(index).items():
            if len(rows) == 1:
                base[uid] = torch.tensor(0.0)
            else:
                sc = torch.tensor([scores[i] for i in rows])
                ln = torch.tensor([lengths[i] for i in rows])
                base[uid] = (ln * sc).sum() / ln.sum()
        for i in range(scores.shape[0]):
            scores[i] = scores[i] - base[index[i]]
        scores = scores.unsqueeze(-1) * response_mask
    return scores, scores


def compute_reinforce_plus_plus_outcome_advantage(token_level_rewards, response_mask, gamma):
    """trainer/ppo/core_algos.py:533-569 — discounted return, reset after EOS, then whitening."""
    with torch.no_grad():
        returns = torch.zeros_like(token_level_rewards)
        running = 0
        for t in reversed(range(token_level_rewards.shape[1])):
            running = token_level_rewards[:, t] + gamma * running
            returns[:, t] = running
            running = running * response_mask[:, t]
        adv = masked_whiten(returns, response_mask) * response_mask
    return adv, returns


def compute_remax_outcome_advantage(token_level_rewards, reward_baselines, response_mask):
    """trainer/ppo/core_algos.py:572-605."""
    with torch.no_grad():
        returns = (token_level_rewards * response_mask).flip(dims=[-1]).cumsum(dim=-1).flip(dims=[-1])
        adv = returns - reward_baselines.unsqueeze(-1) * response_mask
    return adv, returns


def compute_gpg_outcome_advantage(token_level_rewards, response_mask, index, epsilon=1e-6, f_norm=1.0):
    """trainer/ppo/core_algos.py:608-667 — alpha = B / max(#nonzero scores, 1)."""
    scores = token_level_rewards.sum(dim=-1)
    with torch.no_grad():
        alpha = scores.shape[0] / torch.count_nonzero(scores).clamp(min=1)
        means = {}
        for uid, rows in _groups(index).items():
            members = [scores[i] for i in rows]
            means[uid] = torch.tensor(0.0) if len(members) == 1 else torch.mean(torch.tensor(members))
        for i in range(scores.shape[0]):
            scores[i] = alpha * (scores[i] - means[index[i]]) / f_norm
        scores = scores.unsqueeze(-1) * response_mask
    return scores, scores


def compute_policy_loss_gpg(log_prob, advantages, response_mask, loss_agg_mode="token-mean"):
    """trainer/ppo/core_algos.py:797-815."""
    return agg_loss(-log_prob * advantages, response_mask, loss_agg_mode)


def compute_policy_loss_kl_cov(old_log_prob, log_prob, advantages, response_mask, loss_agg_mode="token-mean",
                               kl_cov_ratio=0.0002, ppo_kl_coef=1.0):
    """trainer/ppo/core_algos.py:908-972 — the top kl_cov_ratio covariance tokens get an |kl| penalty."""
    nkl = log_prob - old_log_prob
    ratio = torch.exp(nkl)
    ppo_kl_abs = masked_mean(nkl.abs(), response_mask)
    pg1 = -advantages * ratio
    pgkl = -advantages * ratio + ppo_kl_coef * nkl.abs()
    pg = pg1
    valid = response_mask > 0
    valid_idx = torch.nonzero(valid.reshape(-1), as_tuple=True)[0]
    a = advantages[valid].detach().reshape(-1)
    lp = log_prob[valid].detach().reshape(-1)
    if min(kl_cov_ratio, len(a)) != 0:
        cov = (a - a.mean()) * (lp - lp.mean())
        k = max(1, int(len(cov) * kl_cov_ratio))
        top = torch.topk(cov, k, largest=True).indices
        if len(top):
            flat = valid_idx[top]
            R = advantages.shape[1]
            pg[flat // R, flat % R] = pgkl[flat // R, flat % R]
    return agg_loss(pg, response_mask, loss_agg_mode), ppo_kl_abs


def compute_gae_advantage_return(token_level_rewards, values, response_mask, gamma, lam):
    """trainer/ppo/core_algos.py:193-241 — masked reverse recurrence; observation tokens
    (mask 0) carry the value and the running advantage through unchanged."""
    with torch.no_grad():
        next_value = 0
        running = 0
        out = []
        for t in reversed(range(token_level_rewards.shape[-1])):
            m = response_mask[:, t]
            delta = token_level_rewards[:, t] + gamma * next_value - values[:, t]
            candidate = delta + gamma * lam * running
            next_value = values[:, t] * m + (1 - m) * next_value
            running = candidate * m + (1 - m) * running
            out.append(running)
        adv = torch.stack(out[::-1], dim=1)
        ret = adv + values
        adv = masked_whiten(adv, response_mask)
    return adv, ret


def apply_kl_penalty(token_level_scores, old_log_probs, ref_log_prob, response_mask, beta, kl_type="kl"):
    """trainer/ppo/ray_trainer.py:153-193 (tensor part): returns (token_level_rewards, current_kl)."""
    kld = kl_penalty(old_log_probs, ref_log_prob, kl_type) * response_mask
    rewards = token_level_scores - beta * kld
    current_kl = torch.mean(masked_mean(kld, mask=response_mask, axis=-1), dim=0).item()
    return rewards, current_kl


def compute_response_mask(responses, attention_mask):
    """trainer/ppo/ray_trainer.py:196-211."""
    return attention_mask[:, -responses.size(1):]


def group_ids(index) -> np.ndarray:
    """Integer group id per row, in first-appearance order (test helper)."""
    order = {}
    return np.array([order.setdefault(u, len(order)) for u in index], dtype=np.int64)
