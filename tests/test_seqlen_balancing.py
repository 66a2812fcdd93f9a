"""Sequence-length balancing: the native Karmarkar-Karp partitioner against
the oracle restatement, the reference's own seqlen-balancing tests
(tests/utils/test_seqlen_balancing.py), dynamic micro-batching, _balance_batch and the DAPO
group filter. CPU only (host code)."""

import os
import random

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle.seqlen_balancing_ref import karmarkar_karp as kk_oracle
from verl_amd.protocol import DataProto
from verl_amd.utils.model import create_random_mask
from verl_amd.utils.seqlen_balancing import (
    ceildiv,
    get_reverse_idx,
    get_seqlen_balanced_partitions,
    greedy_partition,
    karmarkar_karp,
    log_seqlen_unbalance,
    prepare_dynamic_batch,
    rearrange_micro_batches,
    restore_dynamic_batch,
)


def test_kk_known_answer():
    # the largest-differencing example {8,7,6,5,4}, k=2: sums 16 / 14
    parts = karmarkar_karp([8, 7, 6, 5, 4], 2, equal_size=False)
    assert parts == [[4, 1, 3], [0, 2]]
    assert sorted(sum([8, 7, 6, 5, 4][i] for i in p) for p in parts) == [14, 16]


def test_kk_native_matches_oracle():
    rng = random.Random(0)
    for _ in range(400):
        k = rng.randint(1, 9)
        eq = rng.random() < 0.5
        n = rng.randint(1, 8) * k if eq else rng.randint(k, 70)
        # mixes of ties, zeros and long tails
        vals = [rng.choice([rng.randint(0, 4), rng.randint(1, 3000), 7]) for _ in range(n)]
        assert karmarkar_karp(vals, k, eq) == kk_oracle(vals, k, eq), (vals, k, eq)


def test_kk_headline_sizes_match_oracle():
    rng = np.random.default_rng(1)
    vals = rng.integers(64 + 128, 256 + 1024, size=512).tolist()
    assert karmarkar_karp(vals, 8, True) == kk_oracle(vals, 8, True)
    assert karmarkar_karp(vals, 64, False) == kk_oracle(vals, 64, False)


def test_balanced_partitions_contract():
    vals = [5, 1, 9, 3, 3, 7, 2, 8]
    parts = get_seqlen_balanced_partitions(vals, 4, equal_size=True)
    assert all(p == sorted(p) and len(p) == 2 for p in parts)
    assert sorted(i for p in parts for i in p) == list(range(8))
    with pytest.raises(AssertionError):
        get_seqlen_balanced_partitions([1, 2], 3, equal_size=False)
    with pytest.raises(AssertionError):
        karmarkar_karp([1, 2, 3], 2, equal_size=True)


def test_greedy_partition_known_answer():
    # input order, lightest partition first (lowest index on ties)
    assert greedy_partition([5, 1, 4, 2], 2, equal_size=False) == [[0, 3], [1, 2]]  # 5 | 1, 4 | tie -> 0
    parts = greedy_partition([5, 1, 4, 2], 2, equal_size=True)
    assert [len(p) for p in parts] == [2, 2]


def test_log_seqlen_unbalance():
    vals = [10, 1, 1, 10]
    m = log_seqlen_unbalance(vals, [[0, 1], [2, 3]], "g")
    assert m["g/min"] == 11 and m["g/max"] == 11 and m["g/mean"] == 11
    m = log_seqlen_unbalance([10, 10, 1, 1], [[0, 2], [1, 3]], "g")
    assert m["g/minmax_diff"] == 18 and m["g/balanced_min"] == 11 and m["g/balanced_max"] == 11


def _proto(bs=20, seed=0):
    np.random.seed(seed)
    torch.manual_seed(seed)
    input_ids = torch.randint(low=0, high=10, size=(bs, 100))
    attention_mask = create_random_mask(input_ids=input_ids, max_ratio_of_left_padding=0.1,
                                        max_ratio_of_valid_token=0.9, min_ratio_of_valid_token=0.5)
    return DataProto.from_single_dict({"input_ids": input_ids, "attention_mask": attention_mask})


def test_seqlen_balancing_roundtrip():
    """tests/utils/test_seqlen_balancing.py:30-46."""
    dp = _proto()
    micro, idx_lists = rearrange_micro_batches(dp.batch, max_token_len=300)
    for m in micro:
        assert int(m["attention_mask"].sum()) <= 300 or len(m["attention_mask"]) == 1
    cat = {k: torch.cat([m[k] for m in micro]) for k in ("input_ids", "attention_mask")}
    flat = [i for ix in idx_lists for i in ix]
    rev = torch.tensor(get_reverse_idx(flat))
    for k in cat:
        torch.testing.assert_close(cat[k][rev], dp.batch[k])
    # largest attention work first
    w = [sum(int(s) ** 2 for s in m["attention_mask"].sum(1)) for m in micro]
    assert w == sorted(w, reverse=True)


def test_dynamic_batch_roundtrip():
    """tests/utils/test_seqlen_balancing.py:49-61."""
    dp = _proto(seed=3)
    dp.non_tensor_batch["uid"] = np.array([f"u{i}" for i in range(len(dp))], dtype=object)
    micro, idx_lists = prepare_dynamic_batch(dp, max_token_len=300)
    ids = torch.cat([m.batch["input_ids"] for m in micro], dim=0)
    torch.testing.assert_close(restore_dynamic_batch(ids, idx_lists), dp.batch["input_ids"])
    uids = np.concatenate([m.non_tensor_batch["uid"] for m in micro])
    assert list(uids[get_reverse_idx([i for ix in idx_lists for i in ix])]) == list(dp.non_tensor_batch["uid"])


def test_dataproto_split_uneven():
    """tests/utils/test_seqlen_balancing.py:125-183."""
    input_ids = torch.randint(low=0, high=10, size=(10, 5))
    dp = DataProto.from_single_dict({"input_ids": input_ids, "attention_mask": torch.ones(10, 5),
                                     "labels": np.array([f"label_{i}" for i in range(10)], dtype=object)})
    splits = dp.split(3)
    assert [len(s) for s in splits] == [3, 3, 3, 1]
    back = DataProto.concat(splits)
    torch.testing.assert_close(back.batch["input_ids"], input_ids)
    np.testing.assert_array_equal(back.non_tensor_batch["labels"], dp.non_tensor_batch["labels"])
    assert len(dp.split(10)) == 1 and len(dp.split(15)) == 1


def _dist_worker(rank, world, port, max_token_len, same_dp, min_mb):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(42 + rank)
        np.random.seed(42 + rank)
        input_ids = torch.randint(0, 10, (20 + rank * 5, 100))
        am = create_random_mask(input_ids=input_ids, max_ratio_of_left_padding=0.1, max_ratio_of_valid_token=0.9,
                                min_ratio_of_valid_token=0.5)
        batch = DataProto.from_single_dict({"input_ids": input_ids, "attention_mask": am}).batch
        micros, idx_lst = rearrange_micro_batches(batch, max_token_len=max_token_len, dp_group=dist.group.WORLD,
                                                  same_micro_num_in_dp=same_dp, min_num_micro_batch=min_mb)
        local = min(len(am), ceildiv(int(am.sum()), max_token_len))
        if min_mb is not None:
            assert len(micros) == max(local, min_mb)
        if same_dp:
            t = torch.tensor([float(local)])
            out = [torch.zeros(1) for _ in range(world)]
            dist.all_gather(out, t)
            assert len(micros) == max(int(c.item()) for c in out)
        else:
            assert len(micros) == max(local, min_mb or 0)
        flat = torch.cat([m["input_ids"] for m in micros])
        inv = torch.tensor(get_reverse_idx([i for s in idx_lst for i in s]))
        torch.testing.assert_close(flat[inv], batch["input_ids"])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("same_dp,min_mb", [(False, 4), (True, None)])
def test_rearrange_distributed_params(same_dp, min_mb):
    """tests/utils/test_seqlen_balancing.py:64-122, 186-205 on gloo (world 2)."""
    port = 29600 + (7 if same_dp else 3)
    mp.spawn(_dist_worker, args=(2, port, 300, same_dp, min_mb), nprocs=2, join=True)


def test_balance_batch_reorders_for_equal_chunks():
    from verl_amd.trainer.ppo.ray_trainer import balance_batch

    dp = _proto(bs=32, seed=5)
    lens = dp.batch["attention_mask"].sum(1).tolist()
    metrics = {}
    balance_batch(dp, world_size=4, metrics=metrics)
    chunks = [int(c.batch["attention_mask"].sum()) for c in dp.chunk(4)]
    assert max(chunks) - min(chunks) <= max(lens)  # KK bound for equal-size parts
    assert metrics["global_seqlen/balanced_max"] == max(chunks)
    assert metrics["global_seqlen/balanced_min"] == min(chunks)
    assert sorted(dp.batch["attention_mask"].sum(1).tolist()) == sorted(lens)


def test_dapo_filter_groups():
    from verl_amd.trainer.ppo.ray_trainer import filter_groups

    # uid a: rewards {1, 0} (kept), b: {1, 1} (std 0: dropped), c: singleton (kept)
    scores = torch.zeros(5, 4)
    scores[:, -1] = torch.tensor([1.0, 1.0, 0.0, 1.0, 0.5])
    dp = DataProto.from_single_dict({"token_level_rewards": scores,
                                     "uid": np.array(["a", "b", "a", "b", "c"], dtype=object)})
    kept, n_prompts = filter_groups(dp, "seq_final_reward")
    assert n_prompts == 2
    assert list(kept.non_tensor_batch["uid"]) == ["a", "a", "c"]
    torch.testing.assert_close(kept.batch["token_level_rewards"][:, -1], torch.tensor([1.0, 0.0, 0.5]))
