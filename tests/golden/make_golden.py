"""Generate the golden fixtures in tests/golden/ from the oracle (oracle/reference_ops.py).

Config 1 of BASELINE.json (core_algos on a synthetic DataProto batch: 32 responses = 4 prompts
x n=8, response length 256, vocab 32,000) plus small log-prob/entropy cases. The oracle is
pinned by the reference's own known-answer tests (tests/test_oracle_kats.py); these fixtures
freeze its outputs so kernels (GPU tests) and oracle (CPU tests) are checked against the same
numbers. Logits are not stored: they are regenerated from the recorded seed with
torch.Generator (CPU), which is deterministic.

Run: python tests/golden/make_golden.py
"""

from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import reference_ops as ref  # noqa: E402

B, R, N_PROMPTS = 32, 256, 4


def config1_inputs(seed=2024):
    g = torch.Generator().manual_seed(seed)
    lens = torch.randint(16, R + 1, (B,), generator=g)
    mask = (torch.arange(R)[None, :] < lens[:, None]).to(torch.int64)
    rewards = torch.zeros(B, R)
    rewards[torch.arange(B), lens - 1] = torch.bernoulli(torch.full((B,), 0.5), generator=g)
    values = torch.randn(B, R, generator=g)
    new = -torch.rand(B, R, generator=g) * 4
    old = new + torch.randn(B, R, generator=g) * 0.2
    refl = new + torch.randn(B, R, generator=g) * 0.1
    ent = torch.rand(B, R, generator=g) * 6
    perm = torch.randperm(B, generator=g)
    uid = np.array([f"uid-{i // 8}" for i in range(B)])[perm.numpy()]
    return dict(mask=mask, rewards=rewards, values=values, new=new, old=old, ref=refl, ent=ent, uid=uid)


def logits_case(seed, rows, V, scale=2.0):
    g = torch.Generator().manual_seed(seed)
    logits = torch.randn(rows, V, generator=g) * scale
    labels = torch.randint(0, V, (rows,), generator=g)
    return logits, labels


LOGIT_CASES = [  # (name, seed, rows, V, dtype, temperature)
    ("v32000_f32", 11, 16, 32000, "float32", 1.0),
    ("v32000_bf16_t07", 12, 16, 32000, "bfloat16", 0.7),
    ("v151936_bf16", 13, 4, 151936, "bfloat16", 1.0),
]


def build() -> dict:
    x = config1_inputs()
    out = {k: (v.numpy() if isinstance(v, torch.Tensor) else v.astype("U")) for k, v in x.items()}
    m, uid = x["mask"], x["uid"]
    adv, _ = ref.compute_grpo_outcome_advantage(x["rewards"].clone(), m, uid)
    out["grpo_adv"] = adv.numpy()
    adv_ns, _ = ref.compute_grpo_outcome_advantage(x["rewards"].clone(), m, uid, norm_adv_by_std_in_grpo=False)
    out["grpo_nostd_adv"] = adv_ns.numpy()
    for tag, (gamma, lam) in {"g1": (1.0, 1.0), "g099": (0.99, 0.95)}.items():
        a, r = ref.compute_gae_advantage_return(x["rewards"], x["values"], m, gamma, lam)
        out[f"gae_{tag}_adv"] = a.numpy()
        out[f"gae_{tag}_ret"] = r.numpy()
    for agg in ["token-mean", "seq-mean-token-sum", "seq-mean-token-mean", "seq-mean-token-sum-norm"]:
        lp = x["new"].clone().requires_grad_(True)
        loss, met = ref.actor_loss(x["old"], lp, adv, m, clip_ratio=0.2, clip_ratio_high=0.28, loss_agg_mode=agg,
                                   ref_log_prob=x["ref"], kl_loss_type="low_var_kl", kl_loss_coef=0.001)
        loss.backward()
        key = agg.replace("-", "_")
        out[f"loss_{key}_scalars"] = np.array([met["pg_loss"].item(), met["pg_clipfrac"].item(), met["ppo_kl"].item(),
                                               met["pg_clipfrac_lower"].item(), met["kl_loss"].item()], dtype=np.float32)
        out[f"loss_{key}_dlp"] = lp.grad.numpy()
    for kt in ["kl", "abs", "mse", "low_var_kl"]:
        out[f"kl_{kt}"] = ref.kl_penalty(x["new"], x["ref"], kt).numpy()
    for name, seed, rows, V, dt, T in LOGIT_CASES:
        logits, labels = logits_case(seed, rows, V)
        logits = logits.to(getattr(torch, dt))
        z = ref.apply_temperature(logits, T)
        out[f"lp_{name}_labels"] = labels.numpy()
        out[f"lp_{name}_logp"] = ref.logprobs_fp32_math(z, labels).numpy()
        out[f"lp_{name}_entropy"] = ref.entropy_from_logits(z.float()).numpy()
    return out


def main():
    out = build()
    path = os.path.join(HERE, "golden_config1.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.0f} KiB, {len(out)} arrays)")


if __name__ == "__main__":
    main()
