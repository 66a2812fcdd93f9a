"""Data-parallel advantage estimation: each rank computes advantages for its own shard.

The reference computes advantages on the driver over the WHOLE batch (ray_trainer.py:214-291),
after ``_balance_batch`` has reordered it (ray_trainer.py:1204-1205), so a prompt group may
span data-parallel ranks. Sharded over W ranks this stays exact when the batch-global
quantities are exchanged:

  * group estimators (GRPO, Dr.GRPO, RLOO, OPO, pass@k, GPG, RF++-baseline): every rank scores
    its own rows on the device (va_row_scores: unmasked reward sums, plus response lengths for
    OPO), then ONE all-gather moves (uid key, score, length) — 16 bytes per response, 8 KB at
    512 responses — so every rank holds the scores of the whole batch in global row order
    (rank-major, the DP_COMPUTE_PROTO concat order, decorator.py:399-408). The group statistics
    then run on the gathered batch (va_group_coef, members in batch order as the reference's
    dict appends them, core_algos.py:290-291) and each rank writes only its own rows
    (va_broadcast_rows). Results equal a single-process run over the concatenated batch
    whether or not groups are intact. uid values are exchanged as 63-bit keys (blake2b of the
    uid's type and value), so ranks agree on group identity without pickling strings;
  * whitening (GAE, REINFORCE++, RF++-baseline; torch_functional.py:206-223) is batch-global:
    each rank merges its rows' (count, sum, M2) into one fp64 triple on the device, the W
    triples are all-gathered (24 bytes per rank), and every rank merges them in rank order with
    the same kernel, so all ranks apply identical (mean, rstd).
"""

from __future__ import annotations

import hashlib

import numpy as np
import torch

from ... import _lib as L
from ... import kernels as K
from ...protocol import DataProto
from ...utils import comm
from .core_algos import AdvantageEstimator

_GROUP_ESTIMATORS = {
    AdvantageEstimator.GRPO: None,  # (code chosen by norm_adv_by_std_in_grpo)
    AdvantageEstimator.RLOO: L.VA_ADV_RLOO,
    AdvantageEstimator.OPO: L.VA_ADV_OPO,
    AdvantageEstimator.GRPO_PASSK: None,
    AdvantageEstimator.GPG: L.VA_ADV_MEAN_ONLY,
    AdvantageEstimator.REINFORCE_PLUS_PLUS_BASELINE: L.VA_ADV_MEAN_ONLY,
}


def _world(group) -> int:
    return comm.world(group)


def _rank(group) -> int:
    return comm.rank(group)


def _all_gather(t: torch.Tensor, group=None) -> list[torch.Tensor]:
    """all_gather of equal-shape tensors; gloo moves host tensors, RCCL device tensors."""
    return comm.all_gather(t, group)


def uid_keys(index) -> np.ndarray:
    """63-bit key per uid: equal uids give equal keys on every rank (the reference groups by the
    uid value itself, core_algos.py:290; uids are uuid4 strings, ray_trainer.py:1160)."""
    cache: dict = {}
    out = np.empty(len(index), dtype=np.int64)
    for i, u in enumerate(index):
        k = cache.get(u)
        if k is None:
            v = u.item() if isinstance(u, np.generic) else u
            d = hashlib.blake2b(f"{type(v).__name__}:{v}".encode(), digest_size=8).digest()
            k = int.from_bytes(d, "little") >> 1
            cache[u] = k
        out[i] = k
    return out


def gather_row_scores(scores: torch.Tensor, lengths: torch.Tensor | None, index, group=None):
    """All-gather (uid key, score, length) of every rank's rows in rank order.

    Returns (scores_all [N] fp32, lengths_all [N] fp32 | None, keys_all np.int64 [N], row_offset
    of this rank in the global batch). One all-gather of the row counts, one of the payload;
    the keys come back to the host (one sync) for the CSR grouping."""
    dev = scores.device
    B = scores.numel()
    w, r = _world(group), _rank(group)
    keys = uid_keys(index)
    if w == 1:
        return scores, lengths, keys, 0
    sizes = [int(s.item()) for s in _all_gather(torch.tensor([B], dtype=torch.int64, device=dev), group)]
    bmax = max(sizes)
    payload = torch.zeros(bmax, 4, dtype=torch.int32, device=dev)
    payload[:B, 0:2] = torch.from_numpy(keys).view(torch.int32).view(B, 2).to(dev, non_blocking=True)
    payload[:B, 2] = scores.view(torch.int32)
    if lengths is not None:
        payload[:B, 3] = lengths.view(torch.int32)
    parts = _all_gather(payload, group)
    rows = torch.cat([p[:s] for p, s in zip(parts, sizes, strict=True)])
    keys_all = rows[:, 0:2].contiguous().view(torch.int64).view(-1).cpu().numpy()
    scores_all = rows[:, 2].contiguous().view(torch.float32)
    lens_all = rows[:, 3].contiguous().view(torch.float32) if lengths is not None else None
    return scores_all, lens_all, keys_all, sum(sizes[:r])


def outcome_coef_dp(token_level_rewards, response_mask, index, epsilon: float, estimator: int, group=None,
                    check_passk: bool = False):
    """Per-row coefficients a(b) of THIS rank's rows, with the group statistics taken over the
    whole (all-gathered) batch. Returns (coef_local [B], scores_all [N])."""
    K._require_device(token_level_rewards, response_mask)
    if len(index) == 0:
        raise ValueError("no score in prompt index: <empty batch>")
    B = token_level_rewards.shape[0]
    scores, lens = K.row_scores(token_level_rewards, response_mask, lengths=(estimator == L.VA_ADV_OPO))
    scores_all, lens_all, keys_all, off = gather_row_scores(scores, lens, index, group)
    order, offsets, G, gmax = K.group_csr(keys_all, scores.device)
    if check_passk:
        counts = np.bincount(np.unique(keys_all, return_inverse=True)[1].reshape(-1))
        if counts.min() < 2:
            raise ValueError(f"Pass@k requires at least 2 samples per group. Got {int(counts.min())} for group "
                             f"{int(np.argmin(counts))}.")
    coef = K.group_coef(scores_all, lens_all, order, offsets, G, gmax, epsilon, estimator)
    return coef[off : off + B], scores_all


def outcome_advantage_dp(token_level_rewards, response_mask, index, epsilon: float, estimator: int, group=None):
    """adv [B, R] of this rank's rows for a group estimator (GRPO family), batch-global groups."""
    coef, _ = outcome_coef_dp(token_level_rewards, response_mask, index, epsilon, estimator, group,
                              check_passk=estimator in (L.VA_ADV_PASSK, L.VA_ADV_PASSK_NOSTD))
    return K.broadcast_rows(coef, response_mask)


def global_whiten_stats(local_merged: torch.Tensor, group=None) -> torch.Tensor:
    """local (n, sum, M2) fp64[3] on the device -> global fp32 stats {mean, rstd, n, flag}."""
    if _world(group) > 1:
        triples = torch.stack(_all_gather(local_merged.contiguous(), group)).contiguous()
    else:
        triples = local_merged.view(1, 3).contiguous()
    _, stats = torch.ops.verl_amd.whiten_finalize(triples.view(-1), triples.shape[0])
    return stats


def masked_whiten_dp(values, mask, group=None, post_multiply_mask: bool = False):
    """masked_whiten over the union of all ranks' rows."""
    _, merged = K.whiten_stats(values, mask)
    stats = global_whiten_stats(merged, group)
    K._raise_whiten_flag(stats)
    return K.whiten_apply(values, mask, stats, post_multiply_mask=post_multiply_mask)


def compute_gae_advantage_return_dp(token_level_rewards, values, response_mask, gamma, lam, group=None):
    """GAE on this rank's rows; whitening statistics over all ranks (one 24-byte all-gather)."""
    K._require_device(token_level_rewards, values, response_mask)
    m, _ = K._mask(response_mask)
    with torch.no_grad():
        adv_raw, ret, part = torch.ops.verl_amd.gae_scan(K._f32(token_level_rewards), K._f32(values), m,
                                                         float(gamma), float(lam))
        P = L.load().va_gae_partial_count(adv_raw.shape[0])
        local, _ = torch.ops.verl_amd.whiten_finalize(part, P)
        stats = global_whiten_stats(local, group)
        K._raise_whiten_flag(stats)
        adv = torch.ops.verl_amd.whiten_apply(adv_raw, stats, None, False)
    return adv, ret


def check_groups_intact(index, group=None) -> bool:
    """True when no uid appears on more than one rank (diagnostic: the group estimators above are
    exact either way)."""
    w = _world(group)
    if w == 1:
        return True
    # RCCL moves device tensors only: stage the exchange on this rank's GPU under nccl
    dev = comm.comm_device(group)
    keys = torch.from_numpy(np.unique(uid_keys(index))).to(dev)
    n = _all_gather(torch.tensor([keys.numel()], device=dev), group)
    nmax = max(int(x.item()) for x in n)
    pad = torch.full((nmax,), -1, dtype=torch.int64, device=dev)
    pad[: keys.numel()] = keys
    allk = torch.cat([p[: int(c.item())] for p, c in zip(_all_gather(pad, group), n, strict=True)])
    return allk.unique().numel() == allk.numel()


@torch.no_grad()
def agg_loss_dp(loss_mat: torch.Tensor, loss_mask: torch.Tensor, loss_agg_mode: str, group=None) -> torch.Tensor:
    """core_algos.agg_loss (core_algos.py:686-719) over the union of all ranks' rows, as the
    reference's driver computes the actor/entropy metric on the whole batch (ray_trainer.py:
    1224-1228). Each rank reduces its rows to (numerator, denominator) in fp64 and one all-reduce
    sums them: token-mean = sum(x m) / (sum m + 1e-8); seq-mean-token-sum / -token-mean = the mean
    over all rows of the row sums / row means; seq-mean-token-sum-norm = sum(x m) / R."""
    from .core_algos import agg_loss

    if _world(group) == 1:
        return agg_loss(loss_mat, loss_mask, loss_agg_mode)
    x = loss_mat.double() * loss_mask.double()
    m = loss_mask.double()
    if loss_agg_mode == "token-mean":
        num, den = x.sum(), m.sum()
    elif loss_agg_mode == "seq-mean-token-sum":
        num, den = x.sum(-1).sum(), torch.tensor(float(x.shape[0]), dtype=torch.float64, device=x.device)
    elif loss_agg_mode == "seq-mean-token-mean":
        num = (x.sum(-1) / m.sum(-1)).sum()
        den = torch.tensor(float(x.shape[0]), dtype=torch.float64, device=x.device)
    elif loss_agg_mode == "seq-mean-token-sum-norm":
        num, den = x.sum() / loss_mask.shape[-1], torch.ones((), dtype=torch.float64, device=x.device)
    else:
        raise ValueError(f"Invalid loss_agg_mode: {loss_agg_mode}")
    t = comm.all_reduce(torch.stack([num, den]), group=group)
    if loss_agg_mode == "token-mean":
        return (t[0] / (t[1] + 1e-8)).float()
    if loss_agg_mode == "seq-mean-token-sum-norm":
        return t[0].float()
    return (t[0] / t[1]).float()


@torch.no_grad()
def compute_advantage_dp(data: DataProto, adv_estimator, gamma: float = 1.0, lam: float = 1.0, num_repeat: int = 1,
                         norm_adv_by_std_in_grpo: bool = True, config=None, group=None) -> DataProto:
    """ray_trainer.compute_advantage (ray_trainer.py:214-291) on this rank's shard of the batch,
    with the batch-global statistics exchanged across the ranks of ``group``. With one rank it
    is ray_trainer.compute_advantage itself."""
    from . import core_algos
    from .ray_trainer import compute_advantage, compute_response_mask

    if _world(group) == 1:
        return compute_advantage(data, adv_estimator, gamma=gamma, lam=lam, num_repeat=num_repeat,
                                 norm_adv_by_std_in_grpo=norm_adv_by_std_in_grpo, config=config)
    if "response_mask" not in data.batch.keys():
        data.batch["response_mask"] = compute_response_mask(data)
    est = AdvantageEstimator(adv_estimator) if not isinstance(adv_estimator, AdvantageEstimator) else adv_estimator
    rewards = data.batch["token_level_rewards"]
    mask = data.batch["response_mask"]
    index = data.non_tensor_batch.get("uid")
    if est == AdvantageEstimator.GAE:
        adv, ret = compute_gae_advantage_return_dp(rewards, data.batch["values"], mask, gamma, lam, group)
    elif est in (AdvantageEstimator.GRPO, AdvantageEstimator.RLOO, AdvantageEstimator.OPO,
                 AdvantageEstimator.GRPO_PASSK):
        if est == AdvantageEstimator.GRPO:
            code = L.VA_ADV_GRPO if norm_adv_by_std_in_grpo else L.VA_ADV_GRPO_NOSTD
        elif est == AdvantageEstimator.GRPO_PASSK:
            norm = config.get("norm_adv_by_std_in_grpo", True) if config is not None else True
            code = L.VA_ADV_PASSK if norm else L.VA_ADV_PASSK_NOSTD
        else:
            code = _GROUP_ESTIMATORS[est]
        adv = outcome_advantage_dp(rewards, mask, index, 1e-6, code, group)
        ret = adv
    elif est == AdvantageEstimator.GPG:
        coef, scores_all = outcome_coef_dp(rewards, mask, index, 1e-6, L.VA_ADV_MEAN_ONLY, group)
        alpha = scores_all.shape[0] / torch.count_nonzero(scores_all).clamp(min=1)
        adv = K.broadcast_rows(alpha * coef / 1.0, mask)
        ret = adv
    elif est == AdvantageEstimator.REINFORCE_PLUS_PLUS_BASELINE:
        coef, _ = outcome_coef_dp(rewards, mask, index, 1e-6, L.VA_ADV_MEAN_ONLY, group)
        centred = K.broadcast_rows(coef, mask)
        adv = masked_whiten_dp(centred, mask, group, post_multiply_mask=True)
        ret = adv
    elif est == AdvantageEstimator.REINFORCE_PLUS_PLUS:
        ret = K.discounted_returns(rewards, mask, config.gamma, L.VA_RET_RFPP)
        adv = masked_whiten_dp(ret, mask, group, post_multiply_mask=True)
    elif est == AdvantageEstimator.REMAX:  # per-row only: no exchange
        adv, ret = core_algos.compute_remax_outcome_advantage(rewards, data.batch["reward_baselines"], mask)
    else:
        raise ValueError(f"Unknown advantage estimator simply: {est.value}")
    data.batch["advantages"] = adv
    data.batch["returns"] = ret
    return data
