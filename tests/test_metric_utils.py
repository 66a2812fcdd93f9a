"""The fit step's data / timing / throughput metrics (trainer/ppo/metric_utils.py:80-258) on CPU.

Single process: the reference's own expected values (tests/trainer/ppo/test_metric_utils_on_cpu.py:
70-210: score/mean 5.0, rewards/mean 2.5, per-token timings over 6 response / 12 overall tokens,
throughput 300 / 150), plus closed forms of the remaining keys. World size 2 (gloo): each rank
holds half of a batch and the merged metrics equal the single-process metrics of the whole batch,
as the reference's driver computes them (ray_trainer.py:1386-1390); global_token_num is gathered
in rank order; perf/mfu is the same per-rank value at W = 2 as at W = 1 for the same per-rank shard
(it was divided by W over a rank-local token list)."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from verl_amd.protocol import DataProto
from verl_amd.trainer.ppo.metric_utils import (SectionTimer, compute_data_metrics, compute_throughout_metrics,
                                               compute_timing_metrics, global_token_num)
from verl_amd.trainer.ppo.trainer_step import reduce_metrics


def _ref_batch():
    """test_metric_utils_on_cpu.py:74-97."""
    return DataProto.from_dict(tensors={
        "token_level_scores": torch.tensor([[1.0, 2.0], [3.0, 4.0]]),
        "token_level_rewards": torch.tensor([[0.5, 1.0], [1.5, 2.0]]),
        "advantages": torch.tensor([[0.1, 0.2], [0.3, 0.4]]),
        "returns": torch.tensor([[1.1, 1.2], [1.3, 1.4]]),
        "responses": torch.zeros((2, 2)),
        "attention_mask": torch.tensor([[1, 1, 1, 1], [1, 1, 1, 1]]),
        "response_mask": torch.tensor([[1, 1], [1, 1]]),
        "values": torch.tensor([[0.9, 1.0], [1.1, 1.2]]),
    })


def test_reduce_metrics_reference_cases():
    """test_metric_utils_on_cpu.py:37-66."""
    assert reduce_metrics({"loss": [1.0, 2.0, 3.0], "accuracy": [0.0, 0.5, 1.0]}) == {"loss": 2.0, "accuracy": 0.5}
    with np.errstate(all="ignore"), pytest.warns(RuntimeWarning):
        assert np.isnan(reduce_metrics({"empty": []})["empty"])
    assert reduce_metrics({"single": [5.0]})["single"] == 5.0


def test_data_metrics_reference_values_with_and_without_critic():
    m = compute_data_metrics(_ref_batch(), use_critic=True)
    for k in ("critic/score/mean", "critic/rewards/mean", "critic/advantages/mean", "critic/returns/mean",
              "critic/values/mean", "critic/vf_explained_var", "response_length/mean", "prompt_length/mean"):
        assert k in m
    assert m["critic/score/mean"] == pytest.approx(5.0, abs=1e-7)  # reference :112
    assert m["critic/rewards/mean"] == pytest.approx(2.5, abs=1e-7)  # reference :113
    # closed forms of the rest (metric_utils.py:121-170)
    assert (m["critic/score/max"], m["critic/score/min"]) == (7.0, 3.0)
    assert m["critic/advantages/mean"] == pytest.approx(0.25) and m["critic/returns/max"] == pytest.approx(1.4)
    ret = torch.tensor([1.1, 1.2, 1.3, 1.4])
    val = torch.tensor([0.9, 1.0, 1.1, 1.2])
    ev = 1.0 - torch.var(ret - val) / (torch.var(ret) + 1e-5)
    assert m["critic/vf_explained_var"] == pytest.approx(float(ev), abs=1e-5)
    assert m["response_length/mean"] == 2.0 and m["response_length/clip_ratio"] == 1.0
    assert m["prompt_length/mean"] == 2.0 and m["prompt_length/clip_ratio"] == 1.0
    m = compute_data_metrics(_ref_batch(), use_critic=False)
    assert "critic/values/mean" not in m and "critic/vf_explained_var" not in m
    assert "critic/score/mean" in m and "critic/rewards/mean" in m and "response_length/mean" in m


def test_data_metrics_masked_lengths_and_num_turns():
    b = _ref_batch()
    b.batch["attention_mask"] = torch.tensor([[0, 1, 1, 0], [1, 1, 1, 1]])
    b.batch["response_mask"] = torch.tensor([[1, 0], [1, 1]])
    b.non_tensor_batch["__num_turns__"] = np.array([1, 3])
    m = compute_data_metrics(b, use_critic=False)
    assert m["critic/advantages/mean"] == pytest.approx((0.1 + 0.3 + 0.4) / 3)
    assert m["response_length/mean"] == 1.5 and m["response_length/min"] == 1.0
    assert m["response_length/clip_ratio"] == 0.5 and m["prompt_length/clip_ratio"] == 0.5
    assert (m["num_turns/min"], m["num_turns/max"], m["num_turns/mean"]) == (1, 3, 2.0)


def test_timing_metrics_reference_values():
    """test_metric_utils_on_cpu.py:126-175: 2 x (3 prompt + 3 response) tokens."""
    b = DataProto.from_dict(tensors={"responses": torch.zeros((2, 3)),
                                     "attention_mask": torch.ones(2, 6, dtype=torch.long)})
    m = compute_timing_metrics(b, {"gen": 0.5, "ref": 0.3, "values": 0.2})
    assert (m["timing_s/gen"], m["timing_s/ref"], m["timing_s/values"]) == (0.5, 0.3, 0.2)
    assert m["timing_per_token_ms/gen"] == pytest.approx(0.5 * 1000 / 6, abs=1e-5)
    assert m["timing_per_token_ms/ref"] == pytest.approx(0.3 * 1000 / 12, abs=1e-5)
    assert m["timing_per_token_ms/values"] == pytest.approx(0.2 * 1000 / 12, abs=1e-5)


def test_throughput_metrics_reference_values():
    """test_metric_utils_on_cpu.py:178-210."""
    b = DataProto(meta_info={"global_token_num": [100, 200, 300]})
    m = compute_throughout_metrics(b, {"step": 2.0}, n_gpus=1)
    assert (m["perf/total_num_tokens"], m["perf/time_per_step"], m["perf/throughput"]) == (600, 2.0, 300.0)
    assert compute_throughout_metrics(b, {"step": 2.0}, n_gpus=2)["perf/throughput"] == 150.0


def test_section_timer_cpu():
    t = SectionTimer("cpu")
    t.start()
    with t.section("adv"):
        pass
    out = t.read()
    assert set(out) == {"adv", "step"} and 0 <= out["adv"] <= out["step"]


# ------------------------------------------------------------------ world size 2
def _batch(B=6, R=5, P=4, seed=3):
    g = torch.Generator().manual_seed(seed)
    am = torch.cat([(torch.rand(B, P, generator=g) > 0.3).long(), torch.ones(B, R, dtype=torch.long)], 1)
    am[:, P + 2 :] = (torch.rand(B, R - 2, generator=g) > 0.4).long()
    am[0, P:] = 1
    rm = am[:, -R:].clone()
    return DataProto.from_dict(
        tensors={"token_level_scores": torch.randn(B, R, generator=g), "token_level_rewards": torch.randn(B, R, generator=g),
                 "advantages": torch.randn(B, R, generator=g), "returns": torch.randn(B, R, generator=g),
                 "values": torch.randn(B, R, generator=g), "responses": torch.zeros(B, R, dtype=torch.long),
                 "attention_mask": am, "response_mask": rm},
        non_tensors={"__num_turns__": np.arange(B) % 3 + 1})


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _w2_worker(rank, world, port, want_data, want_timing):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    full = _batch()
    mine = full.chunk(world)[rank]
    for use_critic in (True, False):
        got = compute_data_metrics(mine, use_critic=use_critic)
        want = want_data[use_critic]
        assert set(got) == set(want)
        for k in want:
            assert got[k] == pytest.approx(want[k], rel=1e-9, abs=1e-9), k
    timing = {"adv": 0.1 * (rank + 1), "update_actor": 1.0 + rank, "step": 3.0}
    got = compute_timing_metrics(mine, timing)
    for k in want_timing:  # the whole batch's token counts, the slowest rank's times
        assert got[k] == pytest.approx(want_timing[k], rel=1e-12), k
    gtn = global_token_num(mine.batch["attention_mask"])
    assert gtn == full.batch["attention_mask"].sum(-1).tolist()

    # perf/mfu/actor: the same per-rank shard at W = 2 (both ranks hold it) and at W = 1
    from verl_amd.utils.model import qwen2_config
    from verl_amd.utils.flops_counter import FlopsCounter
    from verl_amd.workers.dp_workers import perf_metrics

    fc = FlopsCounter(qwen2_config("tiny"), device_name="MI355X")
    shard = full.chunk(world)[0]
    shard.meta_info["global_token_num"] = global_token_num(shard.batch["attention_mask"])
    assert len(shard.meta_info["global_token_num"]) == len(full)
    w2 = perf_metrics(fc, shard, 0.5, 1, world, "actor")["perf/mfu/actor"]
    one = full.chunk(world)[0]
    one.meta_info["global_token_num"] = one.batch["attention_mask"].sum(-1).tolist()
    w1 = perf_metrics(fc, one, 0.5, 1, 1, "actor")["perf/mfu/actor"]
    assert w2 == pytest.approx(w1, rel=1e-12) and w1 > 0
    bare = _batch().chunk(world)[0]  # no global_token_num: the rank's own tokens, no division
    bare.meta_info = {}
    assert perf_metrics(fc, bare, 0.5, 1, world, "actor")["perf/mfu/actor"] == pytest.approx(w1, rel=1e-12)
    dist.destroy_process_group()


def test_metrics_world2_equal_whole_batch():
    full = _batch()  # single-process values of the whole batch, computed here (no process group)
    want_data = {c: compute_data_metrics(full, use_critic=c) for c in (True, False)}
    want_timing = compute_timing_metrics(full, {"adv": 0.2, "update_actor": 2.0, "step": 3.0})
    mp.spawn(_w2_worker, args=(2, _free_port(), want_data, want_timing), nprocs=2, join=True)


def test_whole_batch_metrics_match_reference_formulas():
    """The fp64 partial-sum form equals the reference's torch expressions on one process."""
    b = _batch()
    m = compute_data_metrics(b, use_critic=True)
    rm = b.batch["response_mask"].bool()
    adv = torch.masked_select(b.batch["advantages"], rm)
    ret = torch.masked_select(b.batch["returns"], rm)
    val = torch.masked_select(b.batch["values"], rm)
    assert m["critic/advantages/mean"] == pytest.approx(float(adv.mean()), rel=1e-6)
    assert m["critic/returns/min"] == pytest.approx(float(ret.min()))
    ev = 1.0 - torch.var(ret - val) / (torch.var(ret) + 1e-5)
    assert m["critic/vf_explained_var"] == pytest.approx(float(ev), rel=1e-5)
    score = b.batch["token_level_scores"].sum(-1)
    assert m["critic/score/mean"] == pytest.approx(float(score.mean()), rel=1e-6)
    rl = b.batch["attention_mask"][:, -5:].sum(-1).float()
    assert m["response_length/clip_ratio"] == pytest.approx(float(torch.eq(rl, 5).float().mean()))


def test_explained_var_without_cancellation_at_large_means():
    """the variances behind vf_explained_var are second moments about the merged mean,
    so returns / values of mean 1e8 and unit spread keep their variance (sumsq - n mean^2 in fp64
    would leave only a few bits of it)."""
    b = _batch(B=8, R=16, seed=5)
    g = torch.Generator().manual_seed(11)
    b.batch["returns"] = 1e8 + torch.randn(8, 16, generator=g, dtype=torch.float64)
    b.batch["values"] = 1e8 + 0.5 * torch.randn(8, 16, generator=g, dtype=torch.float64)
    m = compute_data_metrics(b, use_critic=True)
    rm = b.batch["response_mask"].bool()
    ret = torch.masked_select(b.batch["returns"], rm)
    val = torch.masked_select(b.batch["values"], rm)
    ev = 1.0 - torch.var(ret - val) / (torch.var(ret) + 1e-5)
    assert m["critic/vf_explained_var"] == pytest.approx(float(ev), rel=1e-9)


def test_bench_final_metrics_are_the_reference_reduction():
    """bench.py reports reduce_metrics of the last step's lists (utils/metric/utils.py:23-50: the
    mean, max / min by key name; W = 1 here) and counts the clipped-branch tokens of the timed
    steps as pg_clipfrac x each loss micro-batch's response tokens."""
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from verl_amd.trainer.ppo.trainer_step import reduce_metrics_dp

    m = {"actor/pg_loss": [0.5, 0.1, 0.3], "actor/pg_clipfrac": [0.0, 0.25, 0.5], "actor/pg_clipfrac_lower": [0.0, 0.0, 0.1],
         "perf/max_memory_allocated_gb": 3.0, "actor/lr": 1e-6}
    got = reduce_metrics_dp(dict(m))
    assert got == reduce_metrics(dict(m))
    assert got["actor/pg_loss"] == pytest.approx(0.3) and got["perf/max_memory_allocated_gb"] == 3.0
    rm = torch.ones(6, 4, dtype=torch.long)
    rm[2:4, 2:] = 0  # micro-batch 1 (rows 2-3) holds 4 tokens, the others 8
    batch = DataProto.from_dict(tensors={"response_mask": rm})
    clip = bench.clipped_tokens([m, m], batch, micro=2, dynamic=False)
    assert clip == {"clipped_tokens": round(2 * (0.25 * 4 + 0.5 * 8)), "clipped_lower_tokens": round(2 * 0.1 * 8),
                    "response_tokens": 2 * 20}
    assert bench.clipped_tokens([m], batch, micro=2, dynamic=True) is None


def test_validation_metrics_reference_answers():
    """tests/trainer/ppo/test_metric_utils_on_cpu.py:213-318 (bootstrap_metric, calc_maj_val,
    process_validation_metrics) with the reference's own expectations, and the draws equal to the
    reference's global-RNG sequence for the same seed."""
    import numpy as np

    from verl_amd.trainer.ppo.metric_utils import bootstrap_metric, calc_maj_val, process_validation_metrics

    res = bootstrap_metric([1, 2, 3, 4, 5], subset_size=3, reduce_fns=[np.mean, np.max], n_bootstrap=100, seed=42)
    assert len(res) == 2 and abs(res[0][0] - 3.0) <= 0.3 and 3.5 < res[1][0] < 5.0
    np.random.seed(42)  # the reference's draws (np.random.seed + np.random.choice)
    want = [np.max([[1, 2, 3, 4, 5][i] for i in np.random.choice(5, size=3, replace=True)]) for _ in range(100)]
    assert res[1] == (np.mean(want), np.std(want))
    with pytest.raises(ValueError):
        bootstrap_metric([], subset_size=1, reduce_fns=[np.mean])
    assert calc_maj_val([{"pred": "A", "val": 0.9}, {"pred": "B", "val": 0.8}, {"pred": "A", "val": 0.7}],
                        vote_key="pred", val_key="val") == 0.9
    assert calc_maj_val([{"pred": "A", "val": 0.9}, {"pred": "B", "val": 0.8}, {"pred": "B", "val": 0.7},
                         {"pred": "A", "val": 0.6}], vote_key="pred", val_key="val") in (0.9, 0.8)
    r = process_validation_metrics(["source1", "source1", "source2"], ["prompt1", "prompt1", "prompt2"],
                                   {"score": [0.8, 0.9, 0.7]}, seed=42)
    assert "source1" in r and "source2" in r and abs(r["source1"]["score"]["mean@2"] - 0.85) < 1e-12
    r = process_validation_metrics(["source1"] * 3, ["prompt1"] * 3, {"score": [0.8, 0.9, 0.7], "pred": ["A", "B", "A"]},
                                   seed=42)
    assert "maj@2/mean" in r["source1"]["score"] and "maj@3/mean" in r["source1"]["score"]
