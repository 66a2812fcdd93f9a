"""GRPO actor-update benchmark on MI355X (BASELINE.json metric).

One step = the actor-update hot path on this rank's shard: old-logp forward (compute_log_prob),
GRPO advantages (worker-side, exchanging group statistics when groups span ranks), then
update_policy (forward, fused clipped loss + k3 KL loss, backward, bucketed RCCL gradient
all-reduce, grad clip, AdamW). Workload: Qwen2.5-0.5B architecture (random init), 64 prompts x
n=8 = 512 responses x 1024 tokens, prompts left-padded to 256, vocab 151,936 — configs[1] of
BASELINE.json.

Scaling: by default STRONG — one 512 x 1024 batch is split over the W ranks,
64/W prompts (512/W responses) per rank with the prompt groups intact, as the reference's
DP_COMPUTE_PROTO chunk does (single_controller/base/decorator.py:375-385, normalisation
fsdp_workers.py:174-196). ``--balance`` reorders the batch with the Karmarkar-Karp balancer first
(ray_trainer.py:1064-1079), which splits groups over ranks and exercises the cross-rank GRPO
statistics. ``--scaling weak`` gives every rank its own full 512 x 1024 batch.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
  N > 1 without a launcher: bench.py starts ``torch.distributed.run`` as a CHILD process (before
  any GPU call; no exec) with N ranks on 127.0.0.1 and exits with its return code.
Rank 0 prints ONE JSON line (see the driver contract in the task statement).
"""

from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

# HIP runtime: kernel arguments in device memory (read by the dispatch without a host-memory round
# trip; interleaved same-box A/B: 180.4 / 180.5K vs 179.7 / 179.8K tokens/s at N = 1, 174.0K vs
# 172.8K on the N = 8 per-rank workload, profiles/r02/bench_hip_env_ab.txt). Set before anything
# initialises HIP; the launcher's child ranks inherit it. An explicit setting wins.
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
MFMA_BF16_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA peak (no sparsity)
VOCAB = 151936


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


def pmc_traffic_f1(flops_per_launch: float):
    """HBM-side bytes per launch of the fused lm_head kernel (f1) from the committed PMC passes
    (tools/f1_pmc.sh: FETCH_SIZE x2 + WRITE_SIZE) when they were taken at this launch's shape."""
    import glob

    def newest_first(path):  # profiles/r<NN>[/<pass>]/pmc_f1_product.json: latest round, then latest pass
        parts = os.path.relpath(path, os.path.join(ROOT, "profiles")).split(os.sep)[:-1]
        tag = parts[1] if len(parts) > 1 else ""
        return (parts[0], len(tag), tag)

    paths = glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_f1_product.json")) + glob.glob(
        os.path.join(ROOT, "profiles", "r*", "*", "pmc_f1_product.json"))
    for p in sorted(paths, key=newest_first, reverse=True):
        d = json.load(open(p))
        n, h, v = d["shape"]
        if abs(2.0 * n * v * h - flops_per_launch) <= 1e-6 * flops_per_launch:
            return d["traffic_bytes_per_launch"], os.path.relpath(p, ROOT)
    return None, None


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


def _micro_text(micro: int, pass_rows: int, args) -> str:
    """The loss micro-batch part of config.deviations_from_reference_defaults."""
    if args.dynamic_bsz:
        merged = (f"update passes of up to {args.compute_max_tokens} tokens, each holding several of those "
                  "micro-batches, aggregated one by one by the fused loss kernel (seg_off); "
                  if args.compute_max_tokens else "")
        return (f"use_dynamic_bsz with a {args.dynamic_bsz}-token budget (loss scaled by rows / mini-batch, "
                "dp_actor.py:465-467); " + merged)
    passes = (f"update passes of {pass_rows} responses, each holding {pass_rows // micro} of those micro-batches, "
              "aggregated one by one by the fused loss kernel (seg_rows: the same loss, gradient and "
              "per-micro-batch metric lists as separate passes, tests/test_actor_gpu.py); " if pass_rows > micro
              else "")
    if micro == 8:
        return "none for the loss micro-batch (ppo_micro_batch_size_per_gpu 8, SURVEY §8d); " + passes
    same = ("equal to the reference's at 8 with dense responses (equal token counts per micro-batch); "
            if args.responses == "dense" else
            f"with variable response lengths it weights tokens differently than at 8 (each micro-batch's "
            "token-mean is over its own token count, dp_actor.py:465-470); ")
    return f"ppo_micro_batch_size_per_gpu {micro} (SURVEY §8d: 8): " + same + passes


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong",
                    help="strong: one 512x1024 batch split over the ranks (SURVEY §8e); weak: a full batch per rank")
    ap.add_argument("--balance", action="store_true",
                    help="Karmarkar-Karp balance the batch over ranks first (splits prompt groups across ranks)")
    ap.add_argument("--prompts", type=int, default=64)
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--prompt-len", type=int, default=256)
    ap.add_argument("--response-len", type=int, default=1024)
    ap.add_argument("--micro", type=int, default=8,
                    help="ppo_micro_batch_size_per_gpu: the loss micro-batch (responses; SURVEY §8d: 8)")
    ap.add_argument("--compute-micro", type=int, default=128,
                    help="compute_micro_batch_size_per_gpu: responses per update forward/backward pass, holding "
                         "compute-micro / micro loss micro-batches that the fused loss aggregates one by one "
                         "(capped at the rank's shard)")
    ap.add_argument("--logprob-micro", type=int, default=128, help="log_prob_micro_batch_size_per_gpu")
    ap.add_argument("--dynamic-bsz", type=int, default=0,
                    help="use_dynamic_bsz with this ppo_max_token_len_per_gpu (and log-prob budget); 0 = off")
    ap.add_argument("--compute-max-tokens", type=int, default=0,
                    help="with --dynamic-bsz: compute_max_token_len_per_gpu, tokens per update pass holding several "
                         "token-budget micro-batches (0 = one micro-batch per pass, as the reference)")
    ap.add_argument("--logprob-max-tokens", type=int, default=0,
                    help="with --dynamic-bsz: log_prob_max_token_len_per_gpu of the no-grad old-logp pass (per-token "
                         "results, independent of it; 0 = the --dynamic-bsz budget)")
    ap.add_argument("--pad-multiple", type=int, default=2048,
                    help="round packed micro-batches up to a multiple of this many tokens (pack_pad_multiple)")
    ap.add_argument("--gemm-table", default="default",
                    help="tuned GEMM solution table (verl_amd/tuned/*.csv, 'default', or 'none')")
    ap.add_argument("--model", default="0.5b")
    ap.add_argument("--logprob-inplace-bwd", type=int, default=2, choices=[0, 1, 2],
                    help="1: dlogits over the logits (reference's inplace_backward); 0: fresh buffer (faster stream); "
                         "2: fresh buffer when it fits in HBM, else over the logits")
    ap.add_argument("--old-noise", type=float, default=0.05,
                    help="old_log_probs = recomputed + N(0, s^2) (SURVEY §8d: ratios straddle the clip band)")
    ap.add_argument("--zero", type=int, default=0, choices=[0, 1],
                    help="1: ZeRO-style sharded fp32 master / AdamW state over the ranks (reduce-scatter + all-gather)")
    ap.add_argument("--wgrad-stream", type=int, default=0, choices=[0, 1],
                    help="1: backbone weight gradients + fp32 accumulation on a side stream (wgrad_side_stream)")
    ap.add_argument("--fused-no-grad", type=int, default=1, choices=[0, 1],
                    help="1: the no-grad old-logp pass runs the fused lm_head + log-prob kernel (f1, fused_logprob_no_grad)")
    ap.add_argument("--fused-mlp-no-grad", type=int, default=1, choices=[0, 1],
                    help="1: the no-grad old-logp pass runs gate|up + SwiGLU as one kernel (fused_mlp_no_grad)")
    ap.add_argument("--fused-mlp-train", type=int, default=0, choices=[0, 1],
                    help="1: update passes run gate|up + SwiGLU as one kernel that also writes the projection for "
                         "the backward (fused_mlp_train)")
    ap.add_argument("--fused-qkv", type=int, default=0, choices=[0, 1],
                    help="1: the q|k|v GEMM + bias + RoPE as one kernel in every pass (fused_qkv)")
    ap.add_argument("--f1-after-backbone", type=int, default=1, choices=[0, 1],
                    help="1: the no-grad pass runs every micro-batch's backbone, then the fused lm_head launches back "
                         "to back (fused_lm_head_after_backbone); 0: backbone + lm_head per micro-batch")
    ap.add_argument("--f1-concat", type=int, default=0, choices=[0, 1],
                    help="with --f1-after-backbone 1: one fused lm_head launch over all micro-batches' rows")
    ap.add_argument("--fused-kernels", type=int, default=0, choices=[0, 1],
                    help="1: use_fused_kernels for every pass (the update pass too: fused f1 forward + the fused "
                         "dlogits backward, no [N, V] logits in HBM)")
    ap.add_argument("--no-rmpad", action="store_true")
    ap.add_argument("--no-mixed-precision", action="store_true", help="fp32 weights + autocast instead of bf16/fp32-master")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--cpu-sample-rows", type=int, default=2048,
                    help="response tokens per repetition of the CPU baseline's log-prob fwd+bwd sample")
    ap.add_argument("--cpu-reps", type=int, default=5, help="timed repetitions (after 1 warm-up) of the CPU baseline")
    ap.add_argument("--out", default=None, help="also write the JSON line here")
    ap.add_argument("--dump-state", default=None,
                    help="rank 0 writes an .npz of the fp32 masters before / after (every 997th element, bucket order) and "
                         "metrics: compares runs at different world sizes (tests/test_rehearsal_w8_gpu.py)")
    ap.add_argument("--tune", action="append", default=[],
                    help="KEY=VALUE va_set_tuning override for A/B runs (e.g. 8=0: grid-stride SwiGLU)")
    ap.add_argument("--launcher-check", action="store_true",
                    help="only start the ranks, check the world size, run the cross-rank replica check on a "
                         "small CPU module and print a JSON line (no GPU work)")
    ap.add_argument("--responses", choices=["dense", "realistic"], default="dense",
                    help="response lengths: dense (all R valid) or realistic (U[128, R], SURVEY §8d)")
    return ap.parse_args(argv)


_T0 = time.perf_counter()


def log(rank, msg):
    if rank == 0:
        print(f"[bench +{time.perf_counter() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int, argv: list[str]) -> int:
    """Start ``torch.distributed.run`` with n ranks as a child process and return its exit code.

    Called before anything touches the GPU (no HIP initialisation in this parent, and no exec):
    the ranks are fresh processes. A failing rank makes torch.distributed.run exit non-zero."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def cpu_baseline(args) -> dict:
    """The oracle (eager PyTorch CPU restatement of the reference, `port`) timed on the box's host
    cores: BASELINE.md §2 / SURVEY §8d — 1 warm-up + median of ``cpu_reps`` repetitions of
      * log-prob + entropy forward AND backward through autograd over the full vocab for
        ``cpu_sample_rows`` response tokens (fp32 row loop, torch_functional.py:116-133, 145-149;
        the headline's 524,288 x 151,936 logits cannot be materialised on a host, so this is a
        bounded sample scaled per token);
      * GRPO advantages + clipped loss + k3 KL forward/backward over the full 512 x 1024 batch
        (core_algos.py:246-308, 722-794, 1034-1069).
    Reported as hot-path tokens/s (model GEMMs excluded: they are not in the oracle)."""
    import numpy as np
    import torch

    from oracle import reference_ops as ref

    affinity = len(os.sched_getaffinity(0))
    quota, quota_src = cgroup_cpu_quota()
    env_threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or None
    V = VOCAB
    rows = args.cpu_sample_rows
    g = torch.Generator().manual_seed(0)
    logits = torch.randn(rows, V, generator=g) * 2
    labels = torch.randint(0, V, (rows,), generator=g)
    B, R, n = args.prompts * args.n, args.response_len, args.n
    rewards = torch.zeros(B, R)
    rewards[:, -1] = torch.randint(0, 2, (B,), generator=g).float()
    mask = torch.ones(B, R, dtype=torch.int64)
    index = np.array([f"p{i // n}" for i in range(B)], dtype=object)
    new = -torch.rand(B, R, generator=g)
    old = new + 0.05 * torch.randn(B, R, generator=g)
    refl = new + 0.1 * torch.randn(B, R, generator=g)

    def lp_pass():
        x = logits.clone().requires_grad_(True)
        t0 = time.perf_counter()
        lp = ref.logprobs_from_logits(x, labels)
        ent = ref.entropy_from_logits(x)
        (lp.sum() + ent.sum()).backward()
        dt = time.perf_counter() - t0
        del x, lp, ent
        return dt

    def algo_pass():
        t0 = time.perf_counter()
        adv, _ = ref.compute_grpo_outcome_advantage(rewards, mask, index)
        newr = new.clone().requires_grad_(True)
        loss, _ = ref.actor_loss(old, newr, adv, mask, ref_log_prob=refl, kl_loss_type="low_var_kl")
        loss.backward()
        return time.perf_counter() - t0

    def measure(threads):
        torch.set_num_threads(threads)
        lp_pass()  # warm-up
        algo_pass()
        t_lp = sorted(lp_pass() for _ in range(args.cpu_reps))[args.cpu_reps // 2]
        t_algo = sorted(algo_pass() for _ in range(args.cpu_reps))[args.cpu_reps // 2]
        return t_lp, t_algo, 1.0 / (t_lp / rows + t_algo / (B * R))

    # thread counts (the affinity count): the CPU quota of the cgroup bounds what
    # the threads can actually run on; when there is no quota, or one above the box's
    # OMP_NUM_THREADS share, the affinity count is timed as planned AND that share, both reported
    if quota is not None and quota <= affinity:
        plans = [("cgroup_quota", max(1, int(quota)))]
    else:
        plans = [("affinity", affinity)]
        if env_threads and env_threads < affinity:
            plans.append(("omp_num_threads", env_threads))
    runs = []
    for label, threads in plans:
        t_lp, t_algo, v = measure(threads)
        runs.append({"threads": threads, "basis": label, "value": round(v, 1),
                     "median_logprob_s": round(t_lp, 3), "median_algos_s": round(t_algo, 3)})
    best = max(runs, key=lambda r: r["value"])
    return {
        "value": best["value"],
        "unit": "tokens/s",
        "cores": best["threads"],
        "kind": "port",
        "os_cpu_count": os.cpu_count(),
        "affinity_cpus": affinity,
        "cgroup_cpu_quota": quota,
        "cgroup_cpu_quota_source": quota_src,
        "omp_num_threads_env": env_threads,
        "torch_threads": torch.get_num_threads(),
        "runs": runs,
        "sample": (f"oracle log-prob+entropy fwd+bwd (autograd) of {rows} tokens x V={V} fp32 "
                   f"+ GRPO adv + clipped loss + k3 KL fwd/bwd on {B}x{R}; 1 warm-up + median of {args.cpu_reps} "
                   f"per thread count; value = the faster thread count (runs lists each); model GEMMs excluded"),
    }


def clipped_tokens(step_metrics: list, batch, micro: int, dynamic: bool):
    """Tokens on the clipped branches over the timed steps: sum over every loss micro-batch of
    pg_clipfrac (and pg_clipfrac_lower) x its response tokens. The update walks the rank's rows in
    order in micro-batches of ``micro`` rows (dp_actor.update_policy: one mini-batch per rank), so
    the k-th entry of a metric list is rows [k micro, (k+1) micro). None with dynamic micro-batches."""
    if dynamic or not step_metrics:
        return None
    rm = batch.batch["response_mask"]
    B = rm.shape[0]
    per_mb = [float(rm[r:r + micro].sum()) for r in range(0, B, micro)]  # one host sync, after the timed region
    out = {"pg_clipfrac": 0.0, "pg_clipfrac_lower": 0.0}
    for m in step_metrics:
        for key in out:
            vals = m.get(f"actor/{key}", [])
            out[key] += sum(v * per_mb[k % len(per_mb)] for k, v in enumerate(vals))
    return {"clipped_tokens": round(out["pg_clipfrac"]), "clipped_lower_tokens": round(out["pg_clipfrac_lower"]),
            "response_tokens": round(sum(per_mb)) * len(step_metrics)}


def cgroup_cpu_quota():
    """CPUs the process's cgroup may use (cpu.max quota / period, v2; cfs_quota_us / cfs_period_us,
    v1), or None without a quota; with the file it came from."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, p = open(path).read().split()[:2]
            return (None if q == "max" else int(q) / int(p)), f"{path}: {q} {p}"
        except (OSError, ValueError):
            pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return (None if q < 0 else q / p), f"cgroup v1 cfs_quota_us {q} cfs_period_us {p}"
    except (OSError, ValueError):
        return None, "no cgroup cpu quota file readable"


def master_sample(worker):
    """Every 997th element of the fp32 master weights over the buckets in bucket order (padding
    dropped; ZeRO shards all-gathered first, so every rank must call this)."""
    import torch

    from verl_amd.utils import comm

    mgr = worker.actor.grad_reducer
    parts = []
    for i, b in enumerate(mgr.buckets):
        n_real = sum(p.numel() for p in b.params)
        if hasattr(mgr, "shards"):
            full = torch.empty(b.buf.numel(), dtype=torch.float32, device=b.buf.device)
            comm.all_gather_into(full, mgr.shards[i].detach(), mgr.group)
        else:
            full = mgr.master_bufs[i]
        parts.append(full[:n_real][::997].detach().cpu())
    return torch.cat(parts)


def dump_state(path: str, init, worker, metrics, rank: int):
    """rank 0 writes the master samples before the first and after the last step, and the final
    metrics (comparison of world sizes, tests/test_rehearsal_w8_gpu.py)."""
    import numpy as np

    final = master_sample(worker)
    if rank == 0:
        m = metrics.meta_info["metrics"] if metrics is not None else {}
        np.savez(path, masters_init=init.numpy(), masters=final.numpy(),
                 **{k.replace("/", "__"): np.asarray(v, dtype=np.float64) for k, v in m.items()
                    if isinstance(v, (list, float, int))})


def shard_batch(args, rank: int, world: int, dev):
    """This rank's DataProto shard of the benchmark batch.

    strong: the SAME 512 x 1024 batch is built on every rank (seeded), in prompt-group order, and
    rank r takes rows [r B/W, (r+1) B/W) — 64/W whole prompt groups — then shuffles them (the
    permutation _balance_batch would apply inside a rank). With ``balance`` the whole batch is
    first shuffled and KK-balanced over the W ranks (groups split across ranks).
    weak: every rank builds its own full batch (seed 1234 + rank)."""
    import numpy as np
    import torch

    from verl_amd.trainer.ppo.ray_trainer import balance_batch
    from verl_amd.utils.synthetic import make_grpo_batch

    dense = args.responses == "dense"
    if args.scaling == "weak":
        return make_grpo_batch(args.prompts, args.n, args.prompt_len, args.response_len, seed=1234 + rank,
                               device=dev, dense_responses=dense, min_response=128, step_noise=True)
    full = make_grpo_batch(args.prompts, args.n, args.prompt_len, args.response_len, seed=1234,
                           permute=args.balance, dense_responses=dense, min_response=128, step_noise=True)
    B = len(full)
    if B % world:
        raise SystemExit(f"{B} responses do not split evenly over {world} ranks")
    if args.balance:
        balance_batch(full, world, {})
        shard = full.chunk(world)[rank]
    else:
        shard = full.chunk(world)[rank]
        shard.reorder(torch.from_numpy(np.random.RandomState(1234 + rank).permutation(len(shard))))
    return shard.to(dev)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # not under a launcher: start one (child process, before any GPU call) and exit with its rc
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

    import torch
    import torch.distributed as dist

    from verl_amd.workers.dp_workers import init_distributed, local_device_index

    if args.launcher_check:
        os.environ.setdefault("VA_DIST_BACKEND", "gloo")
    rank, world = init_distributed()
    world_seen = dist.get_world_size() if dist.is_initialized() else 1
    if world_seen != args.gpus:
        print(f"[bench] rank {rank}: --gpus {args.gpus} but the process group has {world_seen} ranks",
              file=sys.stderr, flush=True)
        sys.exit(3)
    if args.launcher_check:
        fail = os.environ.get("VA_BENCH_FAIL_RANK")
        if fail is not None and int(fail) == rank:
            print(f"[bench] rank {rank}: failing on request (VA_BENCH_FAIL_RANK)", file=sys.stderr, flush=True)
            sys.exit(7)
        t = torch.tensor([rank + 1.0])
        if world > 1:
            dist.all_reduce(t)
        # the end-of-run replica check on a small CPU model (same seed on every rank);
        # VA_BENCH_PERTURB_RANK changes one rank's weights after the "update" to prove it fires
        from verl_amd.utils.replica_check import replica_check

        torch.manual_seed(0)
        mod = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.Linear(32, 4))
        perturb = os.environ.get("VA_BENCH_PERTURB_RANK")
        if perturb is not None and int(perturb) == rank:
            with torch.no_grad():
                mod[1].weight[0, 0] += 1e-3
        rc = replica_check(mod, None, {"actor/grad_norm": [1.5]}, ["actor/grad_norm"], 0.25)
        if rank == 0:
            print(json.dumps({"launcher_check": True, "n_gpus": args.gpus, "world_seen": world_seen,
                              "rank_sum": float(t.item()), **rc}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        if not rc["replicas_identical"]:
            sys.exit(4)
        return

    from verl_amd import kernels as K
    from verl_amd.trainer.ppo.core_algos import AdvantageEstimator
    from verl_amd.trainer.ppo.metric_utils import global_token_num
    from verl_amd.utils import comm as vcomm
    from verl_amd.utils.config import AttrDict, actor_config
    from verl_amd.utils.model import build_qwen2
    from verl_amd.workers.dp_workers import ActorWorker

    local = local_device_index()
    if args.tune:
        from verl_amd import _lib as L

        for kv in args.tune:
            key, val = (int(x) for x in kv.split("="))
            L.call("va_set_tuning", key, val)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    strong = args.scaling == "strong"
    B_total = args.prompts * args.n * (1 if strong else world)
    B = B_total // world if strong else args.prompts * args.n  # responses on this rank
    R = args.response_len
    micro = min(args.micro, B)
    cmicro = max(micro, min(args.compute_micro, B))
    lp_micro = min(args.logprob_micro, B)
    cfg = AttrDict(
        actor=actor_config(
            # prompts per mini-batch; x rollout_n / world in ActorWorker -> one optimizer step per rank
            ppo_mini_batch_size=args.prompts if strong else args.prompts * world,
            ppo_micro_batch_size_per_gpu=micro,
            compute_micro_batch_size_per_gpu=cmicro,
            use_kl_loss=True, kl_loss_coef=0.001, kl_loss_type="low_var_kl",
            clip_ratio=0.2, clip_ratio_c=3.0, loss_agg_mode="token-mean", entropy_coeff=0,
            use_remove_padding=not args.no_rmpad,
            use_dynamic_bsz=args.dynamic_bsz > 0, ppo_max_token_len_per_gpu=args.dynamic_bsz or 16384,
            compute_max_token_len_per_gpu=args.compute_max_tokens or None,
            pack_pad_multiple=args.pad_multiple,
            logprob_inplace_backward={0: False, 1: True, 2: "auto"}[args.logprob_inplace_bwd],
            fused_logprob_no_grad=bool(args.fused_no_grad),
            fused_mlp_no_grad=bool(args.fused_mlp_no_grad),
            fused_mlp_train=bool(args.fused_mlp_train),
            fused_qkv=bool(args.fused_qkv),
            fused_lm_head_after_backbone=bool(args.f1_after_backbone),
            fused_lm_head_concat=bool(args.f1_concat),
            use_fused_kernels=bool(args.fused_kernels),
            wgrad_side_stream=bool(args.wgrad_stream),
            gemm_tuning_file=None if args.gemm_table in (None, "none") else args.gemm_table,
        ),
        rollout=AttrDict(log_prob_micro_batch_size_per_gpu=lp_micro, temperature=1.0,
                         log_prob_use_dynamic_bsz=args.dynamic_bsz > 0,
                         log_prob_max_token_len_per_gpu=args.logprob_max_tokens or args.dynamic_bsz or 16384),
    )
    worker = ActorWorker(cfg, rollout_n=args.n)
    model = build_qwen2(args.model, device=dev, seed=0)
    worker.init_model(model, mixed_precision=not args.no_mixed_precision, zero=bool(args.zero))
    log(rank, f"model ready ({sum(p.numel() for p in model.parameters()) / 1e6:.1f}M params), world={world}, "
              f"{args.scaling} scaling, {B} responses on this rank")
    init_sample = master_sample(worker) if args.dump_state else None
    batch = shard_batch(args, rank, world, dev)
    assert len(batch) == B, (len(batch), B)
    # the whole batch's per-sequence token counts (ray_trainer.py:1208), gathered over the ranks
    batch.meta_info["global_token_num"] = global_token_num(batch.batch["attention_mask"])
    # reference-policy log-probs are an input of the step (ref = new + N(0, 0.1^2)); the
    # N(0, 1) draws are per row of the global batch (make_grpo_batch step_noise), so the step's
    # inputs do not depend on the number of ranks
    old_noise = batch.batch.pop("old_noise")
    ref_noise = batch.batch.pop("ref_noise")
    with torch.no_grad():
        lp0 = worker.compute_log_prob(batch).batch["old_log_probs"]
        batch.batch["ref_log_prob"] = lp0 + 0.1 * ref_noise
    del lp0, ref_noise

    def step():
        out = worker.compute_log_prob(batch)
        old = out.batch["old_log_probs"]
        if args.old_noise:
            # old = new + N(0, 0.05^2) so the timed step exercises the clip branches
            old = old + args.old_noise * old_noise
        batch.batch["old_log_probs"] = old
        worker.compute_advantage(batch, AdvantageEstimator.GRPO, norm_adv_by_std_in_grpo=True)
        return worker.update_actor(batch)

    log(rank, "batch + reference log-probs ready")
    for i in range(args.warmup):
        step()
        torch.cuda.synchronize()
        log(rank, f"warmup step {i} done")
    torch.cuda.synchronize()
    if not args.no_kernel_timing:
        K.TIMER = K.KernelTimer()
    comm_timer = worker.actor.grad_reducer.start_timing() if world > 1 else None
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    prof_path = os.environ.get("VA_BENCH_CPROFILE")  # host-side profile of the timed steps (diagnostics)
    prof = None
    if prof_path and rank == 0:
        import cProfile

        prof = cProfile.Profile()
        prof.enable()
    from verl_amd import custom_ops

    fallbacks0 = custom_ops.AUTO_INPLACE_FALLBACKS
    tprof_path = os.environ.get("VA_BENCH_TORCH_PROFILE")  # where the step's aten ops come from (diagnostics)
    tprof = None
    if tprof_path and rank == 0:
        tprof = torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU], with_stack=True)
        tprof.__enter__()
    t0 = time.perf_counter()
    metrics = None
    step_metrics = []  # each timed step's metric lists (host values: update_actor returns them)
    for i in range(args.steps):
        metrics = step()
        step_metrics.append(metrics.meta_info["metrics"])
        log(rank, f"timed step {i} issued")
    torch.cuda.synchronize()
    if tprof is not None:
        tprof.__exit__(None, None, None)
        with open(tprof_path, "w") as f:
            f.write(tprof.key_averages(group_by_stack_n=6).table(sort_by="count", row_limit=40, max_name_column_width=40))
    if prof is not None:
        prof.disable()
        prof.dump_stats(prof_path)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    lp_fallbacks = custom_ops.AUTO_INPLACE_FALLBACKS - fallbacks0
    t = torch.tensor([elapsed, -elapsed], dtype=torch.float64, device=dev)
    vcomm.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, fastest = float(t[0].item()), -float(t[1].item())
    ksum = K.TIMER.summary() if K.TIMER is not None else {}
    K.TIMER = None
    comm = None
    if world > 1:
        exposed_ms = worker.actor.grad_reducer.stop_timing()
        ex = torch.tensor([exposed_ms / args.steps], dtype=torch.float64, device=dev)
        vcomm.all_reduce(ex, op=dist.ReduceOp.MAX)
        comm = {"exposed_allreduce_ms_per_step": round(float(ex.item()), 3),
                "isolated_allreduce_ms_per_step": round(worker.actor.grad_reducer.time_isolated_sync(), 3),
                "grad_bytes": worker.actor.grad_reducer.grad_bytes(),
                "backend": dist.get_backend()}
    del comm_timer

    resp_tokens = torch.tensor([int(batch.batch["response_mask"].sum().item())], dtype=torch.float64, device=dev)
    vcomm.all_reduce(resp_tokens)
    tok_s = float(resp_tokens.item()) * args.steps / elapsed
    # metric_utils.py:249-257: the whole batch's tokens per second per GPU
    perf_throughput = sum(batch.meta_info["global_token_num"]) * args.steps / elapsed / world

    log(rank, f"timed region: {elapsed:.2f}s for {args.steps} steps")
    # the reference's reduction of the last step's metric lists (utils/metric/utils.py:23-50: mean,
    # max / min by key name), then over the ranks as its DP collect does; and the clipped-branch
    # token counts of all timed steps, summed over the ranks
    from verl_amd.trainer.ppo.trainer_step import reduce_metrics_dp

    final_metrics = reduce_metrics_dp(dict(metrics.meta_info["metrics"])) if metrics is not None else {}
    clip = clipped_tokens(step_metrics, batch, micro, args.dynamic_bsz > 0)
    if clip is not None and world > 1:
        ct = torch.tensor([clip[k] for k in sorted(clip)], dtype=torch.float64, device=dev)
        vcomm.all_reduce(ct)
        clip = {k: round(float(v)) for k, v in zip(sorted(clip), ct.tolist())}
    # after the timed region: every rank must hold the same model (FSDP's by-construction
    # consistency, fsdp_workers.py:370-405) and the same globally-reduced metrics
    from verl_amd.utils.replica_check import replica_check

    rcheck = replica_check(worker.module, worker.actor.grad_reducer,
                           metrics.meta_info["metrics"] if metrics is not None else {},
                           ["actor/grad_norm", "actor/lr"], elapsed - fastest)
    log(rank, f"replica check: {rcheck}")
    if args.dump_state:
        dump_state(args.dump_state, init_sample, worker, metrics, rank)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:  # the contract: rank 0 at N = 1 only
        cpu = cpu_baseline(args)
        log(rank, f"cpu baseline: {cpu['value']} tokens/s on {cpu['cores']} threads")

    if rank == 0:
        roof_hbm = roof_f1 = None
        # the rooflines are the §8 path's kernels (the log-prob kernels, f1); the model-side
        # kernels the timer also records (weight_grad, adamw_flat) are reported under `kernels` only
        hbm = {k: v for k, v in ksum.items() if "tflops" not in v and k.startswith("logprob_entropy")}
        if hbm:
            # the streaming log-prob kernels: the dominant HBM-bound one by time
            name, d = max(hbm.items(), key=lambda kv: kv[1]["time_ms_total"])
            traffic, src = pmc_traffic(name, d["avg_bytes"], VOCAB)
            per_row = 2 * 2 * VOCAB + 28 if name.endswith("bwd") else 2 * VOCAB + 20  # bf16 rows
            ceil, ceil_src = hbm_ceiling(name, round(d["avg_bytes"] / per_row),
                                         args.logprob_inplace_bwd == 1 or lp_fallbacks > 0)
            roof_hbm = {
                "kernel": name, "bound": "hbm", "achieved": round(d["gbps"], 1), "peak": HBM_PEAK_GBPS,
                "unit": "GB/s", "frac": round(d["gbps"] / HBM_PEAK_GBPS, 4),
                "traffic": round(traffic) if traffic else None, "traffic_source": src,
                "measured_stream_ceiling": ceil,
                "frac_of_measured_ceiling": round(d["gbps"] / ceil, 4) if ceil else None,
                "ceiling_source": ceil_src, "algo_bytes_per_launch": d["avg_bytes"],
                "avg_launch_us": round(d["avg_us"], 2), "launches": d["launches"],
                "time_ms_total": round(d["time_ms_total"], 2),
            }
        f1s = {k: v for k, v in ksum.items() if "tflops" in v and k.startswith("linear_logprob")}
        if f1s:  # MFMA-bound fused lm_head kernels (f1): 2 N V H flops per launch, the dominant one by time
            name, f1 = max(f1s.items(), key=lambda kv: kv[1]["time_ms_total"])
            f1_traffic, f1_src = pmc_traffic_f1(f1["avg_flops"]) if name == "linear_logprob_fwd" else (None, None)
            roof_f1 = {
                "kernel": name, "bound": "mfma", "achieved": round(f1["tflops"], 1),
                "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": round(f1["tflops"] / MFMA_BF16_PEAK_TFLOPS, 4),
                "traffic": round(f1_traffic) if f1_traffic else None, "traffic_source": f1_src,
                "algo_flops_per_launch": f1["avg_flops"], "avg_launch_us": round(f1["avg_us"], 2),
                "launch_us_min_median_max": [round(f1["min_us"], 1), round(f1["median_us"], 1), round(f1["max_us"], 1)],
                "launches": f1["launches"], "time_ms_total": round(f1["time_ms_total"], 2),
            }
        # `roofline`: the §8 kernel that takes the most time in the timed steps (the fused
        # lm_head + log-prob forward since the old-logp pass runs it); both stay in the line
        cands = [r for r in (roof_hbm, roof_f1) if r is not None]
        roof = max(cands, key=lambda r: r["time_ms_total"]) if cands else None
        line = {
            "metric": "GRPO actor-update tokens/sec (512x1024)",
            "value": round(tok_s, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "world_seen": world_seen,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 2),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (random token ids, Bernoulli outcome rewards; random-init weights)",
            "config": {
                "workload": "GRPO actor update: old-logp fwd + GRPO adv + fwd/fused clipped loss+k3 KL/bwd + "
                            "RCCL grad all-reduce + clip + AdamW",
                "model": "Qwen2.5-0.5B architecture",
                "global_batch": B_total,
                "responses_per_gpu": B,
                "prompts_per_gpu": args.prompts // world if strong else args.prompts,
                "groups_split_over_ranks": bool(args.balance and world > 1 and strong),
                "seq_len": args.prompt_len + R,
                "response_len": R,
                "vocab": VOCAB,
                "micro_batch": micro,
                "compute_micro_batch": worker.actor._pass_rows("vanilla") if not args.dynamic_bsz else None,
                "logprob_micro_batch": lp_micro,
                "old_logp_noise": args.old_noise,
                "response_lengths": (f"dense: all {R} valid" if args.responses == "dense"
                                     else f"realistic: U[128, {R}]"),
                "deviations_from_reference_defaults": (
                    _micro_text(micro, worker.actor._pass_rows("vanilla"), args)
                    + {0: "out-of-place log-prob backward (reference: in place)",
                       1: "in-place log-prob backward as the reference",
                       2: "out-of-place log-prob backward when its dlogits buffer fits in HBM, else in place as the "
                          f"reference ({lp_fallbacks} in-place fallbacks in the timed steps)"}[args.logprob_inplace_bwd]
                    + ("; the no-grad old-logp pass runs the fused lm_head + log-prob kernel (the reference's "
                       "use_fused_kernels option, off by default there; same bf16-rounded logits, tests)"
                       if args.fused_no_grad else "")
                    + ("; the no-grad pass runs gate|up + SwiGLU as one kernel (the [T, 2F] projection never "
                       "reaches HBM; the same bits as the merged GEMM + SwiGLU on exact-arithmetic data, tests, and "
                       "on the bench's data, relative L2 0.0)" if args.fused_mlp_no_grad else "")
                    + ("; the update pass runs gate|up + SwiGLU as one kernel that also writes the projection "
                       "(the same bits, tests)" if args.fused_mlp_train else "")
                    + ("; the q|k|v GEMM, bias and RoPE run as one kernel (tests)" if args.fused_qkv else "")),
                "dynamic_bsz_max_token_len": args.dynamic_bsz or None,
                "compute_max_token_len": args.compute_max_tokens or None,
                "logprob_max_token_len": (args.logprob_max_tokens or args.dynamic_bsz) if args.dynamic_bsz else None,
                "peak_hbm_gb": round(torch.cuda.max_memory_allocated() / 1e9, 1),
                "pack_pad_multiple": args.pad_multiple,
                "logprob_inplace_backward": {0: False, 1: True, 2: "auto"}[args.logprob_inplace_bwd],
                "logprob_bwd_inplace_fallbacks": lp_fallbacks,
                "fused_logprob_no_grad": bool(args.fused_no_grad),
                "fused_mlp_no_grad": bool(args.fused_mlp_no_grad),
                "fused_mlp_train": bool(args.fused_mlp_train),
                "fused_qkv": bool(args.fused_qkv),
                "fused_lm_head_after_backbone": bool(args.f1_after_backbone),
                "fused_lm_head_concat": bool(args.f1_concat),
                "use_fused_kernels": bool(args.fused_kernels),
                "zero_sharded_optimizer": bool(args.zero),
                "wgrad_side_stream": bool(args.wgrad_stream),
                "hip_env": {"HIP_FORCE_DEV_KERNARG": os.environ.get("HIP_FORCE_DEV_KERNARG")},
                "tuning_overrides": args.tune or None,
                "gemm_table": _gemm_table_name(),
                "parallelism": f"dp{world}",
                "remove_padding": not args.no_rmpad,
                "mixed_precision": "bf16 weights / fp32 master+grads+reduce" if not args.no_mixed_precision
                else "fp32 weights + bf16 autocast",
            },
            "perf_throughput": round(perf_throughput, 1),
            "comm": comm,
            "roofline": roof,
            "roofline_f1": roof_f1,
            "roofline_hbm": roof_hbm,
            "kernels": {k: {kk: (round(vv, 3) if isinstance(vv, float) else vv) for kk, vv in v.items()}
                        for k, v in ksum.items()},
            "cpu_baseline": cpu,
            "replicas_identical": rcheck["replicas_identical"],
            "replica_check": rcheck,
            "final_metrics": final_metrics,
            "final_metrics_reduction": "reduce_metrics (utils/metric/utils.py:23-50) of the last timed step, "
                                       "mean over the ranks",
            "clip_branch_tokens_timed_steps": clip,
        }
        s = json.dumps(line)
        print(s, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(s + "\n")
    if world > 1:
        dist.destroy_process_group()
    if not rcheck["replicas_identical"]:
        print(f"[bench] rank {rank}: replicas differ after the run: {rcheck}", file=sys.stderr, flush=True)
        sys.exit(4)


if __name__ == "__main__":
    main()
