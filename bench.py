"""GRPO actor-update benchmark on MI355X (BASELINE.json metric).

One step = the actor-update hot path on this rank's shard: old-logp forward (compute_log_prob),
GRPO advantages, then update_policy (forward, fused clipped loss + k3 KL loss, backward,
bucketed RCCL gradient all-reduce, grad clip, AdamW). Workload per rank: Qwen2.5-0.5B
architecture (random init), 64 prompts x n=8 = 512 responses x 1024 tokens, prompts left-padded
to 256, vocab 151,936 — configs[1] of BASELINE.json; weak scaling (every rank does that work).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
  N > 1 is launched by torch.distributed.run (one process per GPU, RCCL).
Rank 0 prints ONE JSON line (see the driver contract in the task statement).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
MFMA_BF16_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA peak (no sparsity)


def pmc_traffic(kernel: str, algo_bytes_per_launch: float, vocab: int):
    """HBM bytes per launch from the committed rocprofv3 PMC passes (FETCH_SIZE x2 + WRITE_SIZE,
    MI355X_MICROARCH.md §HBM corrections) of the same kernel, scaled to this launch's rows."""
    import glob

    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_logprob*.json")))
    cands = []
    for p in paths:
        d = json.load(open(p))
        k = d["kernels"].get(kernel)
        if k is None or d.get("vocab") != vocab:
            continue
        rows = algo_bytes_per_launch / (k["algo_bytes"] / d["rows_per_launch"])
        cands.append((abs(d["rows_per_launch"] - rows), -len(cands), k, rows, p))
    if not cands:
        return None, None
    # the pass measured at this launch's own row count when there is one (else scaled per row)
    _, _, k, rows, p = min(cands, key=lambda c: (c[0], c[1]))
    return k["traffic_bytes_per_row"] * rows, os.path.relpath(p, ROOT)


def hbm_ceiling(kernel: str, rows: int | None = None, inplace: bool = False):
    """Best plain-streaming rate measured on MI355X at the same footprint (tools/hbm_stream.hip,
    profiles/r*/hbm_stream_<rows>rows.jsonl, the file of the launch's own row count when present):
    read-only for the forward, read+write (in place when the backward writes over its input) for
    the backward."""
    import glob
    import re

    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "hbm_stream_*rows.jsonl")))
    if not paths:
        return None, None

    def nrows(p):
        m = re.search(r"hbm_stream_(\d+)rows", p)
        return int(m.group(1)) if m else 0

    path = min(paths, key=lambda p: (abs(nrows(p) - rows) if rows else 0, -paths.index(p)))
    mode = "read" if kernel.endswith("fwd") else ("copy_inplace" if inplace else "copy")
    recs = [json.loads(line) for line in open(path) if line.startswith("{")]
    best = max((r["gbps"] for r in recs if r["mode"] == mode), default=None)
    return best, os.path.relpath(path, ROOT)


def _gemm_table_name():
    from verl_amd.utils import gemm_tuning

    return os.path.basename(gemm_tuning._loaded) if gemm_tuning._loaded else None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--prompts", type=int, default=64)
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--prompt-len", type=int, default=256)
    ap.add_argument("--response-len", type=int, default=1024)
    ap.add_argument("--micro", type=int, default=128, help="ppo_micro_batch_size_per_gpu (responses)")
    ap.add_argument("--logprob-micro", type=int, default=128, help="log_prob_micro_batch_size_per_gpu")
    ap.add_argument("--dynamic-bsz", type=int, default=0,
                    help="use_dynamic_bsz with this ppo_max_token_len_per_gpu (and log-prob budget); 0 = off")
    ap.add_argument("--pad-multiple", type=int, default=2048,
                    help="round packed micro-batches up to a multiple of this many tokens (pack_pad_multiple)")
    ap.add_argument("--gemm-table", default="default",
                    help="tuned GEMM solution table (verl_amd/tuned/*.csv, 'default', or 'none')")
    ap.add_argument("--model", default="0.5b")
    ap.add_argument("--logprob-inplace-bwd", type=int, default=0,
                    help="1: dlogits over the logits (reference's inplace_backward); 0: fresh buffer (faster stream)")
    ap.add_argument("--no-rmpad", action="store_true")
    ap.add_argument("--no-mixed-precision", action="store_true", help="fp32 weights + autocast instead of bf16/fp32-master")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--cpu-sample-rows", type=int, default=24576,
                    help="response tokens of the CPU baseline's log-prob sample (~10 s on 16 cores)")
    ap.add_argument("--out", default=None, help="also write the JSON line here")
    ap.add_argument("--tune", action="append", default=[],
                    help="KEY=VALUE va_set_tuning override for A/B runs (e.g. 8=0: grid-stride SwiGLU)")
    return ap.parse_args()


_T0 = time.perf_counter()


def log(rank, msg):
    if rank == 0:
        print(f"[bench +{time.perf_counter() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def _barrier(world):
    if world > 1:
        dist.barrier()


def cpu_baseline(args, rank) -> dict | None:
    """Oracle (eager PyTorch CPU restatement of the reference) on the box's host cores, bounded
    sample: log-prob + entropy of ``cpu_sample_rows`` response tokens over the full vocab (fp32
    row loop, torch_functional.py:116-133, 145-149) and GRPO + clipped loss + k3 KL over the
    full 512 x 1024 batch (core_algos.py). Reported as hot-path tokens/s (not the whole update:
    the model GEMMs are outside the oracle)."""
    if rank != 0:
        return None
    from oracle import reference_ops as ref

    # the box grants a CPU share (OMP_NUM_THREADS=16 there) although affinity lists every host CPU
    cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(len(os.sched_getaffinity(0)), 16)
    torch.set_num_threads(cores)
    V = 151936
    chunk = min(args.cpu_sample_rows, 2048)  # one 1.2 GB fp32 logits buffer, reused per chunk
    n_chunks = max(1, args.cpu_sample_rows // chunk)
    rows = chunk * n_chunks
    g = torch.Generator().manual_seed(0)
    logits = torch.randn(chunk, V, generator=g) * 2
    t_lp = 0.0
    for _ in range(n_chunks):
        labels = torch.randint(0, V, (chunk,), generator=g)
        t0 = time.perf_counter()
        lp = ref.logprobs_from_logits(logits, labels)
        ent = ref.entropy_from_logits(logits)
        t_lp += time.perf_counter() - t0
        del lp, ent
    del logits
    B, R, n = args.prompts * args.n, args.response_len, args.n
    rewards = torch.zeros(B, R)
    rewards[:, -1] = torch.randint(0, 2, (B,), generator=g).float()
    mask = torch.ones(B, R, dtype=torch.int64)
    index = np.array([f"p{i // n}" for i in range(B)], dtype=object)
    new = -torch.rand(B, R, generator=g)
    old = new + 0.05 * torch.randn(B, R, generator=g)
    refl = new + 0.1 * torch.randn(B, R, generator=g)
    t0 = time.perf_counter()
    adv, _ = ref.compute_grpo_outcome_advantage(rewards, mask, index)
    newr = new.clone().requires_grad_(True)
    loss, _ = ref.actor_loss(old, newr, adv, mask, ref_log_prob=refl, kl_loss_type="low_var_kl")
    loss.backward()
    t_algo = time.perf_counter() - t0
    per_token = t_lp / rows + t_algo / (B * R)
    return {
        "value": round(1.0 / per_token, 1),
        "unit": "tokens/s",
        "cores": cores,
        "kind": "port",
        "sample": (f"oracle log-prob+entropy fwd of {rows} tokens ({n_chunks} x {chunk}) x V={V} fp32 ({t_lp:.2f}s) + GRPO adv + "
                   f"clipped loss + k3 KL fwd/bwd on {B}x{R} ({t_algo:.2f}s); model GEMMs excluded"),
    }


def main():
    args = parse()
    from verl_amd import kernels as K
    from verl_amd.trainer.ppo.core_algos import AdvantageEstimator
    from verl_amd.trainer.ppo.ray_trainer import compute_advantage
    from verl_amd.utils.config import AttrDict, actor_config
    from verl_amd.utils.model import build_qwen2
    from verl_amd.utils.synthetic import make_grpo_batch
    from verl_amd.workers.dp_workers import ActorWorker, init_distributed, local_device_index

    rank, world = init_distributed()
    local = local_device_index()
    if args.tune:
        from verl_amd import _lib as L

        for kv in args.tune:
            key, val = (int(x) for x in kv.split("="))
            L.call("va_set_tuning", key, val)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world != args.gpus and rank == 0:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)

    B = args.prompts * args.n
    R = args.response_len
    cfg = AttrDict(
        actor=actor_config(
            ppo_mini_batch_size=args.prompts,  # prompts; x n / world in ActorWorker -> one optimizer step
            ppo_micro_batch_size_per_gpu=args.micro,
            use_kl_loss=True, kl_loss_coef=0.001, kl_loss_type="low_var_kl",
            clip_ratio=0.2, clip_ratio_c=3.0, loss_agg_mode="token-mean", entropy_coeff=0,
            use_remove_padding=not args.no_rmpad,
            use_dynamic_bsz=args.dynamic_bsz > 0, ppo_max_token_len_per_gpu=args.dynamic_bsz or 16384,
            pack_pad_multiple=args.pad_multiple,
            logprob_inplace_backward=bool(args.logprob_inplace_bwd),
            gemm_tuning_file=None if args.gemm_table in (None, "none") else args.gemm_table,
        ),
        rollout=AttrDict(log_prob_micro_batch_size_per_gpu=args.logprob_micro, temperature=1.0,
                         log_prob_use_dynamic_bsz=args.dynamic_bsz > 0,
                         log_prob_max_token_len_per_gpu=args.dynamic_bsz or 16384),
    )
    # weak scaling: every rank owns a full 512-response shard; normalise against world=1
    worker = ActorWorker(cfg, rollout_n=args.n * world)
    model = build_qwen2(args.model, device=dev, seed=0)
    worker.init_model(model, mixed_precision=not args.no_mixed_precision)
    log(rank, f"model ready ({sum(p.numel() for p in model.parameters()) / 1e6:.1f}M params), world={world}")
    batch = make_grpo_batch(args.prompts, args.n, args.prompt_len, R, seed=1234 + rank, device=dev)
    # reference-policy log-probs are an input of the step (ref = new + N(0, 0.1^2))
    with torch.no_grad():
        lp0 = worker.compute_log_prob(batch).batch["old_log_probs"]
        gen = torch.Generator(device=dev).manual_seed(99 + rank)
        batch.batch["ref_log_prob"] = lp0 + 0.1 * torch.randn(lp0.shape, device=dev, generator=gen)
    del lp0

    def step():
        out = worker.compute_log_prob(batch)
        batch.batch["old_log_probs"] = out.batch["old_log_probs"]
        compute_advantage(batch, AdvantageEstimator.GRPO, norm_adv_by_std_in_grpo=True)
        return worker.update_actor(batch)

    log(rank, "batch + reference log-probs ready")
    for i in range(args.warmup):
        step()
        torch.cuda.synchronize()
        log(rank, f"warmup step {i} done")
    torch.cuda.synchronize()
    if not args.no_kernel_timing:
        K.TIMER = K.KernelTimer()
    _barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    metrics = None
    for i in range(args.steps):
        metrics = step()
        log(rank, f"timed step {i} issued")
    torch.cuda.synchronize()
    _barrier(world)
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    ksum = K.TIMER.summary() if K.TIMER is not None else {}
    K.TIMER = None

    resp_tokens = int(batch.batch["response_mask"].sum().item())
    total_tokens = torch.tensor([resp_tokens, sum(batch.meta_info["global_token_num"])], dtype=torch.float64,
                                device=dev)
    if world > 1:
        dist.all_reduce(total_tokens)
    tok_s = float(total_tokens[0].item()) * args.steps / elapsed
    perf_throughput = float(total_tokens[1].item()) * args.steps / elapsed / world  # metric_utils.py:249-257

    log(rank, f"timed region: {elapsed:.2f}s for {args.steps} steps")
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:  # the contract: rank 0 at N = 1 only
        cpu = cpu_baseline(args, rank)
        log(rank, f"cpu baseline: {cpu['value']} tokens/s on {cpu['cores']} threads")

    if rank == 0:
        roof = None
        if ksum:
            dom = max(ksum.items(), key=lambda kv: kv[1]["time_ms_total"])
            name, d = dom
            if "tflops" in d:  # MFMA-bound fused lm_head + log-prob kernel
                roof = {
                    "kernel": name,
                    "bound": "mfma",
                    "achieved": round(d["tflops"], 1),
                    "peak": MFMA_BF16_PEAK_TFLOPS,
                    "unit": "TFLOP/s",
                    "frac": round(d["tflops"] / MFMA_BF16_PEAK_TFLOPS, 4),
                    "traffic": None,
                    "algo_flops_per_launch": d["avg_flops"],
                    "avg_launch_us": round(d["avg_us"], 2),
                    "launches": d["launches"],
                }
            else:
                traffic, src = pmc_traffic(name, d["avg_bytes"], 151936)
                per_row = 2 * 2 * 151936 + 28 if name.endswith("bwd") else 2 * 151936 + 20  # bf16 rows
                ceil, ceil_src = hbm_ceiling(name, round(d["avg_bytes"] / per_row), bool(args.logprob_inplace_bwd))
                roof = {
                    "kernel": name,
                    "bound": "hbm",
                    "achieved": round(d["gbps"], 1),
                    "peak": HBM_PEAK_GBPS,
                    "unit": "GB/s",
                    "frac": round(d["gbps"] / HBM_PEAK_GBPS, 4),
                    "traffic": round(traffic) if traffic else None,
                    "traffic_source": src,
                    "measured_stream_ceiling": ceil,
                    "frac_of_measured_ceiling": round(d["gbps"] / ceil, 4) if ceil else None,
                    "ceiling_source": ceil_src,
                    "algo_bytes_per_launch": d["avg_bytes"],
                    "avg_launch_us": round(d["avg_us"], 2),
                    "launches": d["launches"],
                }
        line = {
            "metric": "GRPO actor-update tokens/sec (512x1024)",
            "value": round(tok_s, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (random token ids, Bernoulli outcome rewards; random-init weights)",
            "config": {
                "workload": "GRPO actor update: old-logp fwd + GRPO adv + fwd/fused clipped loss+k3 KL/bwd + "
                            "RCCL grad all-reduce + clip + AdamW",
                "model": "Qwen2.5-0.5B architecture",
                "global_batch": B * world,
                "responses_per_gpu": B,
                "seq_len": args.prompt_len + R,
                "response_len": R,
                "vocab": 151936,
                "micro_batch": args.micro,
                "logprob_micro_batch": args.logprob_micro,
                "dynamic_bsz_max_token_len": args.dynamic_bsz or None,
                "peak_hbm_gb": round(torch.cuda.max_memory_allocated() / 1e9, 1),
                "pack_pad_multiple": args.pad_multiple,
                "logprob_inplace_backward": bool(args.logprob_inplace_bwd),
                "tuning_overrides": args.tune or None,
                "gemm_table": _gemm_table_name(),
                "parallelism": f"dp{world}",
                "remove_padding": not args.no_rmpad,
                "mixed_precision": "bf16 weights / fp32 master+grads+reduce" if not args.no_mixed_precision
                else "fp32 weights + bf16 autocast",
            },
            "perf_throughput": round(perf_throughput, 1),
            "roofline": roof,
            "kernels": {k: {kk: (round(vv, 3) if isinstance(vv, float) else vv) for kk, vv in v.items()}
                        for k, v in ksum.items()},
            "cpu_baseline": cpu,
            "final_metrics": {k: v[-1] for k, v in (metrics.meta_info["metrics"].items() if metrics is not None else [])},
        }
        s = json.dumps(line)
        print(s, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(s + "\n")
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
