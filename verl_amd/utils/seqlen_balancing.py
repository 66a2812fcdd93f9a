"""Sequence-length balancing — mirror of verl/utils/seqlen_balancing.py on MI355X hosts.

Same public functions, arguments and results as the reference; the Karmarkar-Karp partitioner
(seqlen_balancing.py:26-127) runs natively (``va_karmarkar_karp`` in libverl_amd.so, host code,
identical partitions) because it sits in front of every mini-batch when ``use_dynamic_bsz`` is
on. Everything else is small host bookkeeping over index lists.

Used by
  * the trainer's ``_balance_batch`` (ray_trainer.py:1064-1079): equal-size partitions across DP
    ranks so every rank gets a similar token count;
  * the actor's dynamic micro-batching (dp_actor.py:321-347, 382-384, 465-467): micro-batches
    cut by a token budget (``ppo_max_token_len_per_gpu``) instead of a fixed sample count.
"""

from __future__ import annotations

import ctypes
from itertools import chain

import numpy as np
import torch
import torch.distributed as dist

from .. import _lib as L
from ..protocol import DataProto, TensorBatch
from . import comm

__all__ = [
    "karmarkar_karp", "greedy_partition", "get_seqlen_balanced_partitions", "log_seqlen_unbalance", "ceildiv",
    "roundup_divisible", "rearrange_micro_batches", "get_reverse_idx", "prepare_dynamic_batch",
    "restore_dynamic_batch",
]


def karmarkar_karp(seqlen_list: list[int], k_partitions: int, equal_size: bool) -> list[list[int]]:
    """seqlen_balancing.py:26-127 — largest differencing method; partitions in the reference's
    order (not sorted inside)."""
    n = len(seqlen_list)
    if equal_size:
        assert n % k_partitions == 0, f"{n} % {k_partitions} != 0"
    vals = np.ascontiguousarray(np.asarray(seqlen_list, dtype=np.int64).reshape(-1))
    order = np.empty(max(n, 1), dtype=np.int64)
    offsets = np.empty(k_partitions + 1, dtype=np.int64)
    vp = ctypes.c_void_p
    L.call("va_karmarkar_karp", vp(vals.ctypes.data), n, k_partitions, int(bool(equal_size)),
           vp(order.ctypes.data), vp(offsets.ctypes.data))
    parts = [order[offsets[i] : offsets[i + 1]].tolist() for i in range(k_partitions)]
    if equal_size:
        for p in parts:
            assert len(p) * k_partitions == n, f"{len(p)} * {k_partitions} != {n}"
    return parts


def greedy_partition(seqlen_list: list[int], k_partitions: int, equal_size: bool) -> list[list[int]]:
    """seqlen_balancing.py:130-148 — items in input order to the lightest partition (with a bias
    of sum+1 per item under equal_size, so counts balance first)."""
    bias = sum(seqlen_list) + 1 if equal_size else 0
    parts: list[list[int]] = [[] for _ in range(k_partitions)]
    sums = [0] * k_partitions
    for i, v in enumerate(seqlen_list):
        j = min(range(k_partitions), key=lambda t: (sums[t], t))
        parts[j].append(i)
        sums[j] += v + bias
    if equal_size:
        for p in parts:
            assert len(p) * k_partitions == len(seqlen_list), f"{len(p)} * {k_partitions} != {len(seqlen_list)}"
    return parts


def get_seqlen_balanced_partitions(seqlen_list: list[int], k_partitions: int, equal_size: bool):
    """seqlen_balancing.py:151-190 — KK partitions, each checked non-empty and sorted."""
    assert len(seqlen_list) >= k_partitions, f"number of items:[{len(seqlen_list)}] < k_partitions:[{k_partitions}]"
    parts = karmarkar_karp(seqlen_list, k_partitions, equal_size)
    assert len(parts) == k_partitions, f"{len(parts)} != {k_partitions}"
    seen = set()
    out = []
    for i, p in enumerate(parts):
        assert len(p) > 0, f"the {i}-th partition is empty"
        seen.update(p)
        out.append(sorted(p))
    assert seen == set(range(len(seqlen_list)))
    return out


def log_seqlen_unbalance(seqlen_list: list[int], partitions: list[list[int]], prefix):
    """seqlen_balancing.py:193-236 — token sums of the contiguous (pre-balance) chunks vs the
    balanced partitions."""
    k = len(partitions)
    bs = len(seqlen_list) // k
    chunk = [sum(seqlen_list[o : o + bs]) for o in range(0, len(seqlen_list), bs)]
    balanced = [sum(seqlen_list[i] for i in p) for p in partitions]
    return {
        f"{prefix}/min": min(chunk),
        f"{prefix}/max": max(chunk),
        f"{prefix}/minmax_diff": max(chunk) - min(chunk),
        f"{prefix}/balanced_min": min(balanced),
        f"{prefix}/balanced_max": max(balanced),
        f"{prefix}/mean": sum(chunk) / k,
    }


def ceildiv(a, b):
    return -(a // -b)


def roundup_divisible(a, b):
    return ((a + b - 1) // b) * b


def _num_micro_batches(seq_len_effective: list[int], max_token_len: int, dp_group, num_batches_divided_by,
                       same_micro_num_in_dp, min_num_micro_batch, device) -> int:
    total = int(sum(seq_len_effective))
    n = min(len(seq_len_effective), ceildiv(total, max_token_len))
    if min_num_micro_batch is not None:
        n = max(min_num_micro_batch, n)
    if dist.is_available() and dist.is_initialized() and same_micro_num_in_dp:
        t = torch.tensor([n], device=device)
        comm.all_reduce(t, op=dist.ReduceOp.MAX, group=dp_group)
        n = int(t.cpu().item())
    if num_batches_divided_by is not None:
        n = roundup_divisible(n, num_batches_divided_by)
    assert n <= len(seq_len_effective)
    return n


def _collective_device(batch):
    am = batch["attention_mask"]
    if comm.device_backend():
        return am.device if am.is_cuda else comm.comm_device()
    return torch.device("cpu")


def rearrange_micro_batches(batch, max_token_len, dp_group=None, num_batches_divided_by=None,
                            same_micro_num_in_dp=True, min_num_micro_batch=None, use_dynamic_bsz_balance=True):
    """seqlen_balancing.py:239-313 — split by total valid tokens (attention_mask sum) into the
    fewest micro-batches that respect ``max_token_len`` (synchronised to the max over DP ranks),
    balanced by KK; returns (micro-batches, index lists). With ``use_dynamic_bsz_balance`` the
    micro-batches are ordered by decreasing Σ len² (attention work), ties by smallest index."""
    am = batch["attention_mask"]
    max_seq_len = am.shape[-1]
    assert max_token_len >= max_seq_len, (
        f"max_token_len must be greater than the sequence length. Got {max_token_len=} and {max_seq_len=}")
    seq_len_effective = am.sum(dim=1).tolist()
    n = _num_micro_batches(seq_len_effective, max_token_len, dp_group, num_batches_divided_by,
                           same_micro_num_in_dp, min_num_micro_batch, _collective_device(batch))
    parts = get_seqlen_balanced_partitions(seq_len_effective, n, equal_size=False)
    if use_dynamic_bsz_balance:
        parts.sort(key=lambda p: (sum(seq_len_effective[i] ** 2 for i in p), min(p) if p else 0), reverse=True)
    micro = []
    for p in parts:
        idx = torch.as_tensor(p, dtype=torch.long, device=am.device)
        if isinstance(batch, TensorBatch):
            micro.append(TensorBatch({k: v.index_select(0, idx) for k, v in batch.items()}, batch_size=[len(p)]))
        elif isinstance(batch, dict):
            micro.append({k: v.index_select(0, idx) for k, v in batch.items()})
        else:  # a plain tensor
            micro.append(batch.index_select(0, idx))
    return micro, parts


def get_reverse_idx(idx_map):
    """seqlen_balancing.py:316-331 — inverse permutation."""
    rev = list(idx_map)
    for i, j in enumerate(idx_map):
        rev[j] = i
    return rev


def prepare_dynamic_batch(data: DataProto, max_token_len: int) -> tuple[list[DataProto], list[list[int]]]:
    """seqlen_balancing.py:334-353."""
    batches, idx_lists = rearrange_micro_batches(data.batch, max_token_len=max_token_len)
    out = []
    for b, idx in zip(batches, idx_lists, strict=True):
        non_tensors = {k: v[idx] for k, v in data.non_tensor_batch.items()}
        out.append(DataProto(batch=b, non_tensor_batch=non_tensors, meta_info=dict(data.meta_info)))
    return out, idx_lists


def restore_dynamic_batch(data: torch.Tensor, batch_idx_list: list[list[int]]) -> torch.Tensor:
    """seqlen_balancing.py:356-375 — undo the micro-batch permutation."""
    flat = list(chain.from_iterable(batch_idx_list))
    rev = torch.tensor(get_reverse_idx(flat), dtype=torch.long, device=data.device)
    return data[rev]
