"""Drop-in mirror of verl/trainer/ppo/core_algos.py (the PPO/GRPO algorithm layer).

Registries, enum, KL controllers, function names / signatures / defaults and error texts follow
the reference (core_algos.py:33-1069). The hot-path functions run as gfx950 kernels:

  compute_gae_advantage_return     -> va_gae_scan (quad-streaming register scan: one wave per row,
                                      16-B loads, wave-level affine-map scan) + one fused
                                      statistics / whitening launch
  compute_grpo_outcome_advantage   -> va_row_scores -> va_group_coef -> va_broadcast_rows (three
                                      phases: per-row reward sums, per-group fp64 mean / unbiased
                                      std, broadcast a(b) x mask over [B, R])
  compute_rloo_outcome_advantage   -> the same three phases with the RLOO epilogue
  compute_reinforce_plus_plus_baseline_outcome_advantage -> mean-only + whiten kernels
  compute_policy_loss / agg_loss / kl_penalty / compute_entropy_loss -> fused loss kernels

  compute_opo_outcome_advantage / compute_grpo_passk_outcome_advantage -> va_outcome_advantage epilogues
  compute_reinforce_plus_plus_outcome_advantage / compute_remax_outcome_advantage -> va_discounted_returns
  compute_value_loss (critic) -> va_value_loss_fwd/bwd

GPG's advantage reuses the group-mean kernel plus one device-side scale; the gpg / clip_cov /
kl_cov policy-loss variants run in the fused loss kernel (loss modes VA_PL_*); only their
token selection (a batch-global top-k / random subset, not a streaming kernel's shape) is made
with device tensor ops here.
"""

from __future__ import annotations

from enum import Enum
from typing import Optional

import numpy as np
import torch

from ... import _lib as L
from ... import kernels as K
from ...utils import torch_functional as verl_F

__all__ = ["register_adv_est", "get_adv_estimator_fn", "AdvantageEstimator"]

POLICY_LOSS_REGISTRY: dict = {}


def register_policy_loss(name):
    """core_algos.py:36-50."""

    def decorator(func):
        POLICY_LOSS_REGISTRY[name] = func
        return func

    return decorator


def get_policy_loss_fn(name):
    """core_algos.py:53-68."""
    if name not in POLICY_LOSS_REGISTRY:
        raise ValueError(f"Unsupported loss mode: {name}. Supported modes are: {list(POLICY_LOSS_REGISTRY.keys())}")
    return POLICY_LOSS_REGISTRY[name]


ADV_ESTIMATOR_REGISTRY: dict = {}


def register_adv_est(name_or_enum):
    """core_algos.py:74-92."""

    def decorator(fn):
        name = name_or_enum.value if isinstance(name_or_enum, Enum) else name_or_enum
        if name in ADV_ESTIMATOR_REGISTRY and ADV_ESTIMATOR_REGISTRY[name] != fn:
            raise ValueError(f"Adv estimator {name} has already been registered: {ADV_ESTIMATOR_REGISTRY[name]} vs {fn}")
        ADV_ESTIMATOR_REGISTRY[name] = fn
        return fn

    return decorator


def get_adv_estimator_fn(name_or_enum):
    """core_algos.py:95-108."""
    name = name_or_enum.value if isinstance(name_or_enum, Enum) else name_or_enum
    if name not in ADV_ESTIMATOR_REGISTRY:
        raise ValueError(f"Unknown advantage estimator simply: {name}")
    return ADV_ESTIMATOR_REGISTRY[name]


class AdvantageEstimator(str, Enum):
    """core_algos.py:111-128."""

    GAE = "gae"
    GRPO = "grpo"
    REINFORCE_PLUS_PLUS = "reinforce_plus_plus"
    REINFORCE_PLUS_PLUS_BASELINE = "reinforce_plus_plus_baseline"
    REMAX = "remax"
    RLOO = "rloo"
    OPO = "opo"
    GRPO_PASSK = "grpo_passk"
    GPG = "gpg"


class AdaptiveKLController:
    """core_algos.py:131-152 (Ziegler et al. 2019 adaptive KL)."""

    def __init__(self, init_kl_coef, target_kl, horizon):
        self.value = init_kl_coef
        self.target = target_kl
        self.horizon = horizon

    def update(self, current_kl, n_steps):
        err = np.clip(current_kl / self.target - 1, -0.2, 0.2)
        self.value *= 1 + err * n_steps / self.horizon


class FixedKLController:
    """core_algos.py:155-168."""

    def __init__(self, kl_coef):
        self.value = kl_coef

    def update(self, current_kl, n_steps):
        pass


def get_kl_controller(kl_ctrl):
    """core_algos.py:171-190."""
    if kl_ctrl.type == "fixed":
        return FixedKLController(kl_coef=kl_ctrl.kl_coef)
    if kl_ctrl.type == "adaptive":
        assert kl_ctrl.horizon > 0, f"horizon must be larger than 0. Got {kl_ctrl.horizon}"
        return AdaptiveKLController(init_kl_coef=kl_ctrl.kl_coef, target_kl=kl_ctrl.target_kl, horizon=kl_ctrl.horizon)
    raise NotImplementedError


# ==================================================================================== estimators
@register_adv_est(AdvantageEstimator.GAE)
def compute_gae_advantage_return(token_level_rewards, values, response_mask, gamma, lam):
    """core_algos.py:193-241 — returns (whitened advantages, returns)."""
    if token_level_rewards.shape[0] == 0:  # masked_whiten over an empty mask: the reference's ValueError
        raise ValueError("At least one element in the mask has to be 1.")
    with torch.no_grad():
        return K.gae_advantage_return(token_level_rewards, values, response_mask, float(gamma), float(lam))


def _empty_batch(token_level_rewards, response_mask):
    """An empty batch (B = 0): the reference's group loops do not run and it returns the empty
    [0, R] scores x mask (core_algos.py:282-308, 428-530, 311-370), so these estimators return it too
    (the group kernels need B > 0)."""
    if token_level_rewards.shape[0] != 0:
        return None
    empty = torch.zeros(token_level_rewards.shape, dtype=torch.float32, device=token_level_rewards.device)
    return empty * response_mask


@register_adv_est(AdvantageEstimator.GRPO)
def compute_grpo_outcome_advantage(
    token_level_rewards: torch.Tensor,
    response_mask: torch.Tensor,
    index: np.ndarray,
    epsilon: float = 1e-6,
    norm_adv_by_std_in_grpo: bool = True,
    config=None,
) -> tuple[torch.Tensor, torch.Tensor]:
    """core_algos.py:246-308 — GRPO (or Dr.GRPO when norm_adv_by_std_in_grpo is False)."""
    empty = _empty_batch(token_level_rewards, response_mask)
    if empty is not None:
        return empty, empty
    est = L.VA_ADV_GRPO if norm_adv_by_std_in_grpo else L.VA_ADV_GRPO_NOSTD
    with torch.no_grad():
        scores = K.outcome_advantage(token_level_rewards, response_mask, index, epsilon, est)
    return scores, scores


@register_adv_est(AdvantageEstimator.GRPO_PASSK)
def compute_grpo_passk_outcome_advantage(token_level_rewards, response_mask, index, epsilon=1e-6,
                                         norm_adv_by_std_in_grpo=True, config=None, **kwargs):
    """core_algos.py:311-370 — only the best response of each group gets r_max - r_second_max
    (divided by the group's unbiased std + eps when norm_adv_by_std_in_grpo); one group kernel."""
    assert config is not None
    norm = config.get("norm_adv_by_std_in_grpo", True)
    uids, counts = np.unique(np.asarray(index).astype(str), return_counts=True)
    if len(counts) and counts.min() < 2:
        bad = uids[int(np.argmin(counts))]
        raise ValueError(f"Pass@k requires at least 2 samples per group. Got {int(counts.min())} for group {bad}.")
    empty = _empty_batch(token_level_rewards, response_mask)
    if empty is not None:
        return empty, empty
    est = L.VA_ADV_PASSK if norm else L.VA_ADV_PASSK_NOSTD
    with torch.no_grad():
        adv = K.outcome_advantage(token_level_rewards, response_mask, index, epsilon, est)
    return adv, adv


@register_adv_est(AdvantageEstimator.REINFORCE_PLUS_PLUS_BASELINE)
def compute_reinforce_plus_plus_baseline_outcome_advantage(token_level_rewards, response_mask, index, epsilon=1e-6,
                                                           config=None, **kwargs):
    """core_algos.py:376-424: group-mean baseline, then masked whitening, times the mask (an empty
    batch reaches masked_whiten with an all-zero mask: the reference's ValueError)."""
    if token_level_rewards.shape[0] == 0:
        raise ValueError("At least one element in the mask has to be 1.")
    with torch.no_grad():
        # the reference tiles the (s - mean) scalar over all columns before masking: same values
        ones = torch.ones_like(token_level_rewards, dtype=torch.float32)
        centred = K.outcome_advantage(token_level_rewards, ones, index, epsilon, L.VA_ADV_MEAN_ONLY)
        centred = centred * response_mask
        stats, _ = K.whiten_stats(centred, response_mask)
        K._raise_whiten_flag(stats)
        scores = K.whiten_apply(centred, response_mask, stats, post_multiply_mask=True)
    return scores, scores


@register_adv_est(AdvantageEstimator.RLOO)
def compute_rloo_outcome_advantage(token_level_rewards, response_mask, index, epsilon=1e-6, config=None, **kwargs):
    """core_algos.py:428-476 — leave-one-out baseline."""
    empty = _empty_batch(token_level_rewards, response_mask)
    if empty is not None:
        return empty, empty
    with torch.no_grad():
        scores = K.outcome_advantage(token_level_rewards, response_mask, index, epsilon, L.VA_ADV_RLOO)
    return scores, scores


@register_adv_est(AdvantageEstimator.OPO)
def compute_opo_outcome_advantage(token_level_rewards, response_mask, index, epsilon=1e-6, config=None, **kwargs):
    """core_algos.py:479-530 — length-weighted group baseline sum(len*s)/sum(len) (singleton
    groups: baseline 0); one group kernel."""
    empty = _empty_batch(token_level_rewards, response_mask)
    if empty is not None:
        return empty, empty
    with torch.no_grad():
        scores = K.outcome_advantage(token_level_rewards, response_mask, index, epsilon, L.VA_ADV_OPO)
    return scores, scores


@register_adv_est(AdvantageEstimator.REINFORCE_PLUS_PLUS)
def compute_reinforce_plus_plus_outcome_advantage(token_level_rewards, response_mask, config=None, **kwargs):
    """core_algos.py:533-569 — discounted return with reset after EOS (chunked scan kernel), then
    masked whitening (whiten kernels; the reference's ValueErrors), times the mask."""
    assert config is not None
    gamma = config.gamma
    if token_level_rewards.shape[0] == 0:  # masked_whiten over an empty mask: the reference's ValueError
        raise ValueError("At least one element in the mask has to be 1.")
    with torch.no_grad():
        returns = K.discounted_returns(token_level_rewards, response_mask, gamma, L.VA_RET_RFPP)
        stats, _ = K.whiten_stats(returns, response_mask)
        K._raise_whiten_flag(stats)
        advantages = K.whiten_apply(returns, response_mask, stats, post_multiply_mask=True)
    return advantages, returns


@register_adv_est(AdvantageEstimator.REMAX)
def compute_remax_outcome_advantage(token_level_rewards, reward_baselines, response_mask, config=None, **kwargs):
    """core_algos.py:572-605 — reverse cumulative sum of r * mask (scan kernel) minus the
    per-response baseline on valid tokens."""
    empty = _empty_batch(token_level_rewards, response_mask)
    if empty is not None:
        return empty, empty
    with torch.no_grad():
        returns, advantages = K.discounted_returns(token_level_rewards, response_mask, 1.0, L.VA_RET_REMAX,
                                                   baselines=reward_baselines)
    return advantages, returns


@register_adv_est(AdvantageEstimator.GPG)
def compute_gpg_outcome_advantage(token_level_rewards, response_mask, index, epsilon=1e-6, f_norm=1.0, alpha=1.0,
                                  config=None, **kwargs):
    """core_algos.py:608-667: alpha = B / max(#nonzero scores, 1); (s - mean) * alpha / f_norm."""
    empty = _empty_batch(token_level_rewards, response_mask)
    if empty is not None:
        return empty, empty
    scores = token_level_rewards.sum(dim=-1)
    with torch.no_grad():
        alpha = scores.shape[0] / torch.count_nonzero(scores).clamp(min=1)
        centred = K.outcome_advantage(token_level_rewards, torch.ones_like(token_level_rewards), index, epsilon,
                                      L.VA_ADV_MEAN_ONLY)[:, 0]
        scores = (alpha * centred / f_norm).unsqueeze(-1) * response_mask
    return scores, scores


def compute_rewards(token_level_scores, old_log_prob, ref_log_prob, kl_ratio):
    """core_algos.py:670-683."""
    return token_level_scores - (old_log_prob - ref_log_prob) * kl_ratio


# ==================================================================================== losses
_AGG_CODES = K.AGG_MODES


def agg_loss(loss_mat: torch.Tensor, loss_mask: torch.Tensor, loss_agg_mode: str):
    """core_algos.py:686-719."""
    if loss_agg_mode not in _AGG_CODES:
        raise ValueError(f"Invalid loss_agg_mode: {loss_agg_mode}")
    return K.masked_aggregate(loss_mat, loss_mask, _AGG_CODES[loss_agg_mode])


def compute_policy_loss(old_log_prob, log_prob, advantages, response_mask, cliprange=None, cliprange_low=None,
                        cliprange_high=None, clip_ratio_c=3.0, loss_agg_mode: str = "token-mean"):
    """core_algos.py:722-794 — returns (pg_loss, pg_clipfrac, ppo_kl, pg_clipfrac_lower)."""
    lo = cliprange if cliprange_low is None else cliprange_low
    hi = cliprange if cliprange_high is None else cliprange_high
    out = K.fused_policy_loss(old_log_prob, log_prob, advantages, response_mask, lo, hi, clip_ratio_c, loss_agg_mode)
    return out[L.VA_LOSS_PG], out[L.VA_LOSS_CLIPFRAC], out[L.VA_LOSS_PPO_KL], out[L.VA_LOSS_CLIPFRAC_LOWER]


def compute_actor_loss(old_log_prob, log_prob, advantages, response_mask, clip_ratio_low, clip_ratio_high,
                       clip_ratio_c=3.0, loss_agg_mode="token-mean", entropy=None, ref_log_prob=None,
                       kl_loss_type=None, seg_rows=0, seg_off=None):
    """The fused form the actor uses (dp_actor.py:421-461): one kernel for the clipped policy
    loss, the three metrics, agg_loss(kl_penalty) and agg_loss(entropy). Returns the 8-slot
    vector (VA_LOSS_*), or [S, 8] for S loss micro-batches (``seg_rows`` rows each, or the row
    ranges of the ``seg_off`` offsets)."""
    return K.fused_policy_loss(old_log_prob, log_prob, advantages, response_mask, clip_ratio_low, clip_ratio_high,
                               clip_ratio_c, loss_agg_mode, ref_log_prob=ref_log_prob, kl_loss_type=kl_loss_type,
                               entropy=entropy, seg_rows=seg_rows, seg_off=seg_off)


def _variant_loss(old_log_prob, log_prob, advantages, response_mask, loss_agg_mode, mode, selection=None, coef=0.0,
                  clip_lo=0.2, clip_hi=0.2):
    out = K.fused_policy_loss(old_log_prob, log_prob, advantages, response_mask, clip_lo, clip_hi, 3.0, loss_agg_mode,
                              loss_mode=mode, selection=selection, mode_coef=coef)
    return out[L.VA_LOSS_PG], out[L.VA_LOSS_CLIPFRAC], out[L.VA_LOSS_PPO_KL], out[L.VA_LOSS_CLIPFRAC_LOWER]


@register_policy_loss("gpg")
def compute_policy_loss_gpg(old_log_prob, log_prob, advantages, response_mask, loss_agg_mode="token-mean", config=None):
    """core_algos.py:797-815: agg_loss(-log_prob * advantages); the fused loss kernel in mode
    VA_PL_GPG (metric slots 0)."""
    return _variant_loss(old_log_prob, log_prob, advantages, response_mask, loss_agg_mode, "gpg")


@register_policy_loss("clip_cov")
def compute_policy_loss_clip_cov(old_log_prob, log_prob, advantages, response_mask, loss_agg_mode="token-mean",
                                 config=None):
    """core_algos.py:818-905. The token selection (covariance window (lb, ub), tokens not already
    clipped, a random subset of clip_cov_ratio * n_tokens drawn with the reference's
    torch.randperm on the default CPU generator) is made here with device tensor ops; the loss,
    its gradient and the metrics run in the fused kernel (VA_PL_CLIP_COV: max(l1, l2) * corr)."""
    pl = config.policy_loss
    clip_cov_ratio = pl.clip_cov_ratio if pl.clip_cov_ratio is not None else 0.0002
    cliprange = config.clip_ratio
    lo = config.clip_ratio_low if config.clip_ratio_low is not None else cliprange
    hi = config.clip_ratio_high if config.clip_ratio_high is not None else cliprange
    ub = pl.clip_cov_ub if pl.clip_cov_ub is not None else 5.0
    lb = pl.clip_cov_lb if pl.clip_cov_lb is not None else 1.0
    assert clip_cov_ratio > 0, "clip_ratio should be larger than 0."
    with torch.no_grad():
        lp = log_prob.detach()
        ratio = torch.exp(lp - old_log_prob)
        l1 = -advantages * ratio
        l2 = -advantages * torch.clamp(ratio, 1 - lo, 1 + hi)
        clip_by_origin = (l2 > l1) & (response_mask > 0)
        cov_all = (advantages - verl_F.masked_mean(advantages, response_mask)) * (
            lp - verl_F.masked_mean(lp, response_mask))
        cov_all[response_mask == 0] = -torch.inf
        cov_all[clip_by_origin] = -torch.inf
        clip_num = max(int(clip_cov_ratio * response_mask.sum().item()), 1)
        idx = torch.nonzero((cov_all < ub) & (cov_all > lb) & (response_mask > 0))
        if len(idx) > 0:
            perm = torch.randperm(len(idx))
            idx = idx[perm[: min(clip_num, len(idx))].to(idx.device)]
        sel = torch.zeros(advantages.shape, dtype=torch.uint8, device=advantages.device)
        sel[idx[:, 0], idx[:, 1]] = 1
    return _variant_loss(old_log_prob, log_prob, advantages, response_mask, loss_agg_mode, "clip_cov", sel,
                         clip_lo=lo, clip_hi=hi)


@register_policy_loss("kl_cov")
def compute_policy_loss_kl_cov(old_log_prob, log_prob, advantages, response_mask, loss_agg_mode="token-mean",
                               config=None):
    """core_algos.py:908-972. The top-k covariance tokens (k = max(1, int(n_valid * kl_cov_ratio)),
    torch.topk as the reference) are selected here; the loss (-A r + ppo_kl_coef |lp - old| on the
    selection), its gradient and ppo_kl_abs run in the fused kernel (VA_PL_KL_COV)."""
    pl = config.policy_loss
    kl_cov_ratio = pl.kl_cov_ratio if pl.kl_cov_ratio is not None else 0.0002
    ppo_kl_coef = pl.ppo_kl_coef if pl.ppo_kl_coef is not None else 1.0
    assert kl_cov_ratio > 0, "kl_cov_ratio should be larger than 0."
    with torch.no_grad():
        valid = response_mask > 0
        valid_idx = torch.nonzero(valid.reshape(-1), as_tuple=True)[0]
        adv_v = advantages[valid].detach().reshape(-1)
        lp_v = log_prob[valid].detach().reshape(-1)
        sel = torch.zeros(advantages.shape, dtype=torch.uint8, device=advantages.device)
        if min(kl_cov_ratio, len(adv_v)) != 0:
            cov = (adv_v - adv_v.mean()) * (lp_v - lp_v.mean())
            nk = max(1, int(len(cov) * kl_cov_ratio))
            top = torch.topk(cov, nk, largest=True).indices
            if len(top) != 0:
                sel.view(-1)[valid_idx[top]] = 1
    return _variant_loss(old_log_prob, log_prob, advantages, response_mask, loss_agg_mode, "kl_cov", sel,
                         coef=ppo_kl_coef)


def compute_entropy_loss(logits, response_mask, loss_agg_mode: str = "token-mean"):
    """core_algos.py:975-989."""
    token_entropy = verl_F.entropy_from_logits(logits)
    return agg_loss(token_entropy, response_mask, loss_agg_mode)


def compute_value_loss(vpreds, returns, values, response_mask, cliprange_value: float,
                       loss_agg_mode: str = "token-mean"):
    """core_algos.py:992-1031 — clipped value loss (critic), one fused gfx950
    kernel pair (va_value_loss_fwd/bwd). Returns (vf_loss, vf_clipfrac) 0-d fp32 tensors."""
    out = K.fused_value_loss(vpreds, values, returns, response_mask, cliprange_value, loss_agg_mode)
    return out[L.VA_VLOSS_LOSS], out[L.VA_VLOSS_CLIPFRAC]


def kl_penalty(logprob: torch.FloatTensor, ref_logprob: torch.FloatTensor, kl_penalty) -> torch.FloatTensor:
    """core_algos.py:1034-1069: "kl"/"k1", "abs", "mse"/"k2", "low_var_kl"/"k3"; "full" raises."""
    if kl_penalty == "full" or kl_penalty not in K.KL_TYPES:
        raise NotImplementedError
    return K.kl_penalty(logprob, ref_logprob, kl_penalty)


def compute_pf_ppo_reweight_data(data, reweight_method: str = "pow", weight_pow: float = 2.0):
    """core_algos.py:1072-1148 — importance resampling of a DataProto by its scores."""
    from copy import deepcopy

    scores = data.batch["token_level_scores"].sum(dim=-1)
    if reweight_method == "pow":
        w = torch.pow(torch.abs(scores), weight_pow)
    elif reweight_method == "max_min":
        w = torch.where((scores == scores.max()) | (scores == scores.min()), 1.0, 0.0)
    elif reweight_method == "max_random":
        w = torch.where(scores == scores.max(), 0.4, 0.1)
    else:
        raise ValueError(f"Unsupported reweight_method: {reweight_method}")
    w = torch.clamp(w + 1e-8, min=1e-8)
    bs = scores.shape[0]
    idx = torch.multinomial(w, bs, replacement=True)
    idx_np = idx.cpu().numpy()
    out = deepcopy(data)
    from ...protocol import TensorBatch

    out.batch = TensorBatch({k: v[idx] for k, v in data.batch.items()}, batch_size=data.batch.batch_size)
    out.non_tensor_batch = {k: (v[idx_np] if isinstance(v, np.ndarray) else [v[i] for i in idx_np])
                            for k, v in data.non_tensor_batch.items()}
    out.meta_info = {k: ([v[i] for i in idx_np] if isinstance(v, list) and len(v) == bs else v)
                     for k, v in data.meta_info.items()}
    return out
