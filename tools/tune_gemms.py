"""Offline GEMM solution search for the actor's model GEMMs (writes a verl_amd/tuned/*.csv table
that utils/gemm_tuning.use_tuned_gemms loads at run time).

Runs the bench workload (old-logp forward + GRPO update) once per seed with PyTorch TunableOp in
tuning mode, so exactly the GEMM shapes (and bias / transpose variants) the actor issues are
searched. The model uses a small vocabulary: the backbone shapes depend only on the packed token
counts, and the lm_head GEMMs (K = 896, V = 151,936) stay on hipBLASLt's default heuristic.
Seeds 1234..1234+S-1 cover the packed lengths the ranks of a weak-scaling run see.

  python tools/tune_gemms.py --out verl_amd/tuned/gemm_qwen2_0p5b_mi355x.csv --seeds 8 --micro 64 --pad 2048
"""

import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--seeds", type=int, default=8)
    ap.add_argument("--prompts", type=int, default=64)
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--micro", type=int, default=64)
    ap.add_argument("--logprob-micro", type=int, default=64)
    ap.add_argument("--pad", type=int, default=2048)
    ap.add_argument("--vocab", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--duration-ms", type=int, default=30)
    args = ap.parse_args()

    import torch

    from verl_amd.trainer.ppo.core_algos import AdvantageEstimator
    from verl_amd.trainer.ppo.ray_trainer import compute_advantage
    from verl_amd.utils import gemm_tuning
    from verl_amd.utils.config import AttrDict, actor_config
    from verl_amd.utils.model import build_qwen2
    from verl_amd.utils.synthetic import make_grpo_batch
    from verl_amd.workers.dp_workers import ActorWorker, init_distributed

    t0 = time.time()

    def log(msg):
        print(f"[tune +{time.time() - t0:7.1f}s] {msg}", flush=True)

    init_distributed()
    dev = torch.device("cuda", 0)
    cfg = AttrDict(
        actor=actor_config(
            ppo_mini_batch_size=args.prompts, ppo_micro_batch_size_per_gpu=args.micro,
            use_kl_loss=True, kl_loss_coef=0.001, kl_loss_type="low_var_kl", loss_agg_mode="token-mean",
            pack_pad_multiple=args.pad,
        ),
        rollout=AttrDict(log_prob_micro_batch_size_per_gpu=args.logprob_micro, temperature=1.0),
    )
    worker = ActorWorker(cfg, rollout_n=args.n)
    model = build_qwen2("0.5b", device=dev, seed=0, vocab_size=args.vocab)
    worker.init_model(model, mixed_precision=True)
    os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
    gemm_tuning.start_tuning(os.path.abspath(args.out), args.iters, args.duration_ms)
    for s in range(args.seeds):
        batch = make_grpo_batch(args.prompts, args.n, 256, 1024, vocab=args.vocab, seed=1234 + s, device=dev)
        am = batch.batch["attention_mask"]
        log(f"seed {1234 + s}: {int(am.sum())} tokens")
        out = worker.compute_log_prob(batch)
        batch.batch["old_log_probs"] = out.batch["old_log_probs"]
        batch.batch["ref_log_prob"] = out.batch["old_log_probs"] + 0.01
        compute_advantage(batch, AdvantageEstimator.GRPO, norm_adv_by_std_in_grpo=True)
        torch.cuda.synchronize()
        log(f"seed {1234 + s}: log-prob pass tuned")
        worker.update_actor(batch)
        torch.cuda.synchronize()
        log(f"seed {1234 + s}: update tuned")
    gemm_tuning.finish_tuning()
    n = sum(1 for line in open(args.out) if line.startswith("Gemm"))
    log(f"{n} tuned GEMM entries in {args.out}")


if __name__ == "__main__":
    main()
