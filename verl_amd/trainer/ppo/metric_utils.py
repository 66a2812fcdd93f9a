"""The fit step's data / timing / throughput metrics (trainer/ppo/metric_utils.py:50-258, called at
ray_trainer.py:1386-1390), over a batch that is sharded across data-parallel ranks.

The reference computes them on the driver, which holds the whole batch. Here each rank holds its
DP shard on the GPU, so every statistic is formed from per-rank partial sums on the device and
merged over the process group: one fp64 SUM vector (counts, sums, sums of squares) and one MAX
vector (maxima, and minima as negated maxima) per call, then ONE device->host copy. With one rank
the values are the reference's for the same batch (tests/test_metric_utils.py pins them with the
reference's own expected values, tests/trainer/ppo/test_metric_utils_on_cpu.py:98-210).

Timings: the reference times blocking RPCs with host clocks (marked_timer, profiler/performance.py:
156); the step here is asynchronous on the GPU, so ``SectionTimer`` records HIP events on the
compute stream at section boundaries and reads them once at the end of the step, and the
batch-global timing of a section is the slowest rank's (every rank waits for it at the next
exchange).
"""

from __future__ import annotations

import time
from contextlib import contextmanager
from typing import Any

import numpy as np
import torch
import torch.distributed as dist

from ...protocol import DataProto
from ...utils import comm


def _compute_response_info(batch: DataProto) -> dict[str, Any]:
    """metric_utils.py:50-77: response mask, prompt and response lengths from the attention mask."""
    R = batch.batch["responses"].shape[-1]
    am = batch.batch["attention_mask"]
    return dict(response_mask=am[:, -R:], prompt_length=am[:, :-R].sum(-1).float(),
                response_length=am[:, -R:].sum(-1).float())


class _Stats:
    """Named per-rank partial statistics merged in all-reduces (SUM, MAX; then one SUM of the
    second moments about the merged means)."""

    def __init__(self, device):
        self.device = device
        self.sums: list[torch.Tensor] = []
        self.maxs: list[torch.Tensor] = []
        self.sum_idx: dict[str, int] = {}
        self.max_idx: dict[str, int] = {}
        self.moments: list[tuple[str, torch.Tensor]] = []

    def _f64(self, v):
        return v.to(torch.float64).reshape(()) if isinstance(v, torch.Tensor) else \
            torch.tensor(float(v), dtype=torch.float64, device=self.device)

    def add_sum(self, name, v):
        self.sum_idx[name] = len(self.sums)
        self.sums.append(self._f64(v))

    def add_extrema(self, name, x: torch.Tensor):
        """max and min of x (empty -> -inf / +inf, so another rank's values win the merge)."""
        x = x.to(torch.float64).reshape(-1)
        if x.numel():
            hi, lo = x.max(), x.min()
        else:
            hi = lo = torch.tensor(float("inf"), dtype=torch.float64, device=x.device)
            hi = -hi
        self.max_idx[name + "/max"] = len(self.maxs)
        self.maxs.append(hi.to(self.device))
        self.max_idx[name + "/min"] = len(self.maxs)
        self.maxs.append((-lo).to(self.device))

    def add_moments(self, name, x: torch.Tensor):
        """count, sum and extrema of x (fp64); its second moment about the merged mean is formed
        in reduce() (M2 = sum (x - mean)^2, not sumsq - n mean^2: no cancellation when the mean
        is large against the spread)."""
        x = x.to(torch.float64).reshape(-1)
        self.add_sum(name + "/n", x.numel())
        self.add_sum(name + "/sum", x.sum())
        self.moments.append((name, x))
        self.add_extrema(name, x)

    def reduce(self, group=None) -> tuple[dict, dict]:
        dev = comm.comm_device(group) if comm.world(group) > 1 else self.device
        multi = comm.world(group) > 1
        s = torch.stack(self.sums).to(dev) if self.sums else torch.zeros(0, dtype=torch.float64, device=dev)
        m = torch.stack(self.maxs).to(dev) if self.maxs else torch.zeros(0, dtype=torch.float64, device=dev)
        if multi:
            comm.all_reduce(s, group=group)
            comm.all_reduce(m, op=dist.ReduceOp.MAX, group=group)
        # second moments about the batch-global means (still on the device: no host round trip)
        m2 = []
        for name, x in self.moments:
            n = s[self.sum_idx[name + "/n"]]
            mu = s[self.sum_idx[name + "/sum"]] / n.clamp_min(1)
            m2.append(((x.to(dev) - mu) ** 2).sum())
        m2 = torch.stack(m2) if m2 else torch.zeros(0, dtype=torch.float64, device=dev)
        if multi and m2.numel():
            comm.all_reduce(m2, group=group)
        host = torch.cat([s, m, m2]).cpu().tolist()  # the one device->host copy
        sums = {k: host[i] for k, i in self.sum_idx.items()}
        base = len(self.sums) + len(self.maxs)
        for j, (name, _) in enumerate(self.moments):
            sums[name + "/m2"] = host[base + j]
        ext = {}
        for k, i in self.max_idx.items():
            v = host[len(self.sums) + i]
            ext[k] = -v if k.endswith("/min") else v
        return sums, ext


def _mean(s, name):
    n = s[name + "/n"]
    return s[name + "/sum"] / n if n else float("nan")


def _var(s, name):
    """torch.var (unbiased) from the merged count and second moment about the merged mean."""
    n = s[name + "/n"]
    if n < 2:
        return float("nan")
    return s[name + "/m2"] / (n - 1)


def compute_data_metrics(batch: DataProto, use_critic: bool = True, group=None) -> dict[str, Any]:
    """metric_utils.py:80-182 over the union of every rank's rows: score / reward (row sums of the
    token-level tensors), advantages / returns / values over response tokens, vf explained
    variance, response and prompt lengths with their clip ratios, and num_turns when present."""
    tb = batch.batch
    R = tb["responses"].shape[-1]
    dev = tb["attention_mask"].device
    response_mask = tb["response_mask"].bool()
    info = _compute_response_info(batch)
    max_prompt_length = tb["attention_mask"][:, :-R].shape[-1]
    st = _Stats(dev)
    st.add_moments("critic/score", tb["token_level_scores"].sum(-1))
    st.add_moments("critic/rewards", tb["token_level_rewards"].sum(-1))
    valid_adv = torch.masked_select(tb["advantages"], response_mask)
    valid_returns = torch.masked_select(tb["returns"], response_mask)
    st.add_moments("critic/advantages", valid_adv)
    st.add_moments("critic/returns", valid_returns)
    if use_critic:
        valid_values = torch.masked_select(tb["values"], response_mask)
        st.add_moments("critic/values", valid_values)
        st.add_moments("diff", valid_returns - valid_values)
    st.add_moments("response_length", info["response_length"])
    st.add_sum("response_length/clipped", torch.eq(info["response_length"], R).sum())
    st.add_moments("prompt_length", info["prompt_length"])
    st.add_sum("prompt_length/clipped", torch.eq(info["prompt_length"], max_prompt_length).sum())
    turns = batch.non_tensor_batch.get("__num_turns__")
    if turns is not None:
        st.add_moments("num_turns", torch.as_tensor(np.asarray(turns, dtype=np.float64), device=dev))
    s, e = st.reduce(group)

    out: dict[str, Any] = {}
    for name in ("critic/score", "critic/rewards", "critic/advantages", "critic/returns"):
        out[name + "/mean"] = _mean(s, name)
        out[name + "/max"] = e[name + "/max"]
        out[name + "/min"] = e[name + "/min"]
    if use_critic:
        out["critic/values/mean"] = _mean(s, "critic/values")
        out["critic/values/max"] = e["critic/values/max"]
        out["critic/values/min"] = e["critic/values/min"]
        out["critic/vf_explained_var"] = 1.0 - _var(s, "diff") / (_var(s, "critic/returns") + 1e-5)
    for name in ("response_length", "prompt_length"):
        out[name + "/mean"] = _mean(s, name)
        out[name + "/max"] = e[name + "/max"]
        out[name + "/min"] = e[name + "/min"]
        n = s[name + "/n"]
        out[name + "/clip_ratio"] = s[name + "/clipped"] / n if n else float("nan")
    if turns is not None:
        out["num_turns/min"] = e["num_turns/min"]
        out["num_turns/max"] = e["num_turns/max"]
        out["num_turns/mean"] = _mean(s, "num_turns")
    return out


def compute_timing_metrics(batch: DataProto, timing_raw: dict[str, float], group=None) -> dict[str, Any]:
    """metric_utils.py:185-226: timing_s/<section> and timing_per_token_ms/<section> ("gen" per
    response token, ref / values / adv / update_critic / update_actor per prompt+response token),
    token counts over all ranks, each section's time the slowest rank's."""
    info = _compute_response_info(batch)
    keys = sorted(timing_raw)
    if comm.world(group) > 1:
        cdev = comm.comm_device(group)
        tok = torch.stack([info["prompt_length"].double().sum(), info["response_length"].double().sum()]).to(cdev)
        comm.all_reduce(tok, group=group)
        tm = torch.tensor([float(timing_raw[k]) for k in keys], dtype=torch.float64, device=cdev)
        comm.all_reduce(tm, op=dist.ReduceOp.MAX, group=group)
        timing = dict(zip(keys, tm.cpu().tolist(), strict=True))
        num_prompt_tokens, num_response_tokens = tok.cpu().tolist()
    else:
        timing = dict(timing_raw)
        num_prompt_tokens = torch.sum(info["prompt_length"]).item()
        num_response_tokens = torch.sum(info["response_length"]).item()
    num_overall_tokens = num_prompt_tokens + num_response_tokens
    per_section = {"gen": num_response_tokens,
                   **{name: num_overall_tokens for name in ("ref", "values", "adv", "update_critic", "update_actor")}}
    return {
        **{f"timing_s/{name}": value for name, value in timing.items()},
        **{f"timing_per_token_ms/{name}": timing[name] * 1000 / per_section[name]
           for name in set(per_section) & set(timing)},
    }


def compute_throughout_metrics(batch: DataProto, timing_raw: dict[str, float], n_gpus: int) -> dict[str, Any]:
    """metric_utils.py:229-258 (the reference's spelling): ``global_token_num`` lists the valid
    tokens of every sequence of the WHOLE batch (trainer_step gathers it over the ranks, as the
    reference's driver sets it before dispatch, ray_trainer.py:1208); throughput is per GPU."""
    total_num_tokens = sum(batch.meta_info["global_token_num"])
    t = timing_raw["step"]
    return {
        "perf/total_num_tokens": total_num_tokens,
        "perf/time_per_step": t,
        "perf/throughput": total_num_tokens / (t * n_gpus),
    }


class SectionTimer:
    """marked_timer (profiler/performance.py:156-171) for an asynchronous GPU step: HIP events on
    the current stream bracket each section; ``read()`` (after the step's final synchronisation)
    turns them into seconds. ``step`` is the host wall clock from ``start()`` to ``read()``. On a
    CPU device the sections are host clocks."""

    def __init__(self, device):
        self.cuda = torch.device(device).type == "cuda"
        self.marks: dict[str, tuple] = {}
        self.t0 = None

    def start(self):
        self.t0 = time.perf_counter()

    def _mark(self):
        if self.cuda:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            return ev
        return time.perf_counter()

    @contextmanager
    def section(self, name: str):
        a = self._mark()
        try:
            yield
        finally:
            self.marks[name] = (a, self._mark())

    def read(self) -> dict[str, float]:
        if self.cuda:
            torch.cuda.current_stream().synchronize()
        out = {k: (a.elapsed_time(b) / 1e3 if self.cuda else b - a) for k, (a, b) in self.marks.items()}
        out["step"] = time.perf_counter() - self.t0
        return out


def global_token_num(attention_mask: torch.Tensor, group=None) -> list[int]:
    """meta_info["global_token_num"] of the whole batch: every rank's per-sequence valid-token
    counts in rank order (the DP_COMPUTE_PROTO concat order, decorator.py:399-408), so the MFU and
    throughput formulas divide the whole batch's work by the world size as the reference's do
    (fsdp_workers.py:690-697, metric_utils.py:249-257). One all-gather of the row counts and one of
    the padded token counts."""
    local = attention_mask.sum(-1).to(torch.int64)
    if comm.world(group) == 1:
        return local.tolist()
    dev = comm.comm_device(group)
    local = local.to(dev)
    sizes = [int(x.item()) for x in comm.all_gather(torch.tensor([local.numel()], dtype=torch.int64, device=dev), group)]
    pad = torch.zeros(max(sizes), dtype=torch.int64, device=dev)
    pad[: local.numel()] = local
    parts = comm.all_gather(pad, group)
    return torch.cat([p[:n] for p, n in zip(parts, sizes, strict=True)]).tolist()


# ------------------------------------------------------------------ validation metrics (host)
def bootstrap_metric(data: list, subset_size: int, reduce_fns: list, n_bootstrap: int = 1000,
                     seed: int = 42) -> list[tuple[float, float]]:
    """metric_utils.py:261-299: (mean, std) of each reduce_fn over n_bootstrap resamples of
    subset_size items drawn with replacement. The draws are the reference's (MT19937 seeded with
    ``seed``, one choice() per resample), from a local generator instead of the global one."""
    rng = np.random.RandomState(seed)
    per_fn = [[] for _ in reduce_fns]
    for _ in range(n_bootstrap):
        idx = rng.choice(len(data), size=subset_size, replace=True)
        sample = [data[i] for i in idx]
        for out, fn in zip(per_fn, reduce_fns):
            out.append(fn(sample))
    return [(np.mean(v), np.std(v)) for v in per_fn]


def calc_maj_val(data: list[dict], vote_key: str, val_key: str) -> float:
    """metric_utils.py:302-335: the first val_key value of the most frequent vote_key value (ties:
    the vote seen first)."""
    counts, first = {}, {}
    for d in data:
        v = d[vote_key]
        counts[v] = counts.get(v, 0) + 1
        first.setdefault(v, d[val_key])
    return first[max(counts, key=counts.get)]


def process_validation_metrics(data_sources: list[str], sample_inputs: list[str], infos_dict: dict[str, list],
                               seed: int = 42) -> dict:
    """metric_utils.py:338-446: per data source and variable, the mean over prompts of mean@N,
    std@N and, at N = 2, 4, ..., n, the bootstrap best@N / worst@N (and maj@N when a "pred" variable
    exists) of each prompt's responses; string-valued variables are skipped."""
    from collections import defaultdict
    from functools import partial

    groups = defaultdict(lambda: defaultdict(lambda: defaultdict(list)))
    for i, src in enumerate(data_sources):
        for var, vals in infos_dict.items():
            groups[src][sample_inputs[i]][var].append(vals[i])
    collected = defaultdict(lambda: defaultdict(lambda: defaultdict(list)))
    for src, prompts in groups.items():
        for var2vals in prompts.values():
            for var, vals in var2vals.items():
                if isinstance(vals[0], str):
                    continue
                n_resp = len(vals)
                m = {f"mean@{n_resp}": np.mean(vals)}
                if n_resp > 1:
                    m[f"std@{n_resp}"] = np.std(vals)
                    sizes, n = [], 2
                    while n < n_resp:
                        sizes.append(n)
                        n *= 2
                    sizes.append(n_resp)
                    for n in sizes:
                        (b_mean, b_std), (w_mean, w_std) = bootstrap_metric(vals, n, [np.max, np.min], seed=seed)
                        m[f"best@{n}/mean"], m[f"best@{n}/std"] = b_mean, b_std
                        m[f"worst@{n}/mean"], m[f"worst@{n}/std"] = w_mean, w_std
                        if var2vals.get("pred") is not None:
                            votes = [{"val": v, "pred": p} for v, p in zip(vals, var2vals["pred"], strict=True)]
                            [(mj_mean, mj_std)] = bootstrap_metric(
                                votes, n, [partial(calc_maj_val, vote_key="pred", val_key="val")], seed=seed)
                            m[f"maj@{n}/mean"], m[f"maj@{n}/std"] = mj_mean, mj_std
                for name, val in m.items():
                    collected[src][var][name].append(val)
    out = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for src, var2 in collected.items():
        for var, name2 in var2.items():
            for name, vals in name2.items():
                out[src][var][name] = np.mean(vals)
    return out
