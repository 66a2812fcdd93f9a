"""BASELINE config 4 (Qwen2-VL-7B GRPO, multimodal) on the actor-update path.

The reference's _forward_micro_batch takes Qwen2-VL's mrope position ids [bs, 3, S], transposes
them to (3, bs, S) and packs them to (3, 1, nnz) with the tokens (dp_actor.py:106-121), and
feeds the rows' multi_modal_inputs (pixel_values, image_grid_thw; dp_actor.py:89-98) to the
model. Here the packed fused backbone selects the rotary sections itself (qwen2_fused.rotary)
and scatters the model's own vision-tower outputs over the image placeholders
(qwen2_fused.input_embeddings); the HF decoder path (fused_model_ops=False) gets the same
packed (3, 1, T) ids.

Parity: a tiny random-init Qwen2VLForConditionalGeneration (head_dim 64 so the gfx950 flash
kernels run; mrope sections (8, 12, 12)), one image per prompt with get_rope_index's 3-D ids,
compute_log_prob + update_policy against the reference computation (padded HF forward with the
(3, B, S) ids and pixel values + the oracle loss) in float64 and in the reference's own bf16,
with the error budget of tests/test_bench_config_parity_gpu.py (old log-probs placed so that no
token sits within rounding noise of a clip boundary):
  log-probs  max |lp - lp64|         <= 2 max |lp_ref16 - lp64| + 2e-3
  pg_loss    |pg - pg64|             <= 2 |pg_ref16 - pg64| + 1e-4
  gradients  ||g - g64|| / ||g64||   <= 2 (same for ref16) + 1e-3   (all parameters, vision tower too)
The vision tower itself is the HF module (outside SURVEY §8); the BLEU reward of config 4
(custom_reward/bleu_reward.py) is a reward function, outside the actor update.

Qwen2-VL-7B (public card's architecture, random init) runs one GRPO step on one GPU with
property checks, like configs 3 and 5 in test_large_configs_gpu.py.
"""

import copy

import numpy as np
import pytest
import torch

from oracle import reference_ops as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
LOSS = dict(clip_ratio=0.2, loss_agg_mode="token-mean", ref_kl="low_var_kl", kl_coef=0.001)
MB = 4


def _tiny_vl(seed=3):
    from verl_amd.utils.model import build_qwen2_vl

    return build_qwen2_vl("tiny", device=DEV, dtype=torch.float32, seed=seed)


def _params_to(model, dtype):
    for p in model.parameters():
        p.data = p.data.to(dtype)
    return model


def _mm_rows(data, rows):
    mm = data.non_tensor_batch.get("multi_modal_inputs")
    if mm is None:
        return {}
    sel = [mm[i] for i in rows]
    return {"pixel_values": torch.cat([d["pixel_values"] for d in sel]).to(DEV),
            "image_grid_thw": torch.cat([d["image_grid_thw"] for d in sel]).to(DEV)}


def _padded_logits(model, data, rows, dtype=None):
    b = data.batch
    mm = _mm_rows(data, rows)
    if dtype is not None and "pixel_values" in mm:
        mm["pixel_values"] = mm["pixel_values"].to(dtype)
    R = b["responses"].shape[1]
    return model(input_ids=b["input_ids"][rows], attention_mask=b["attention_mask"][rows],
                 position_ids=b["position_ids"][rows].transpose(0, 1), use_cache=False, **mm).logits[:, -R - 1 : -1, :]


def _data(model, images=True, seed=21):
    from verl_amd.utils.synthetic import make_vl_grpo_batch

    data = make_vl_grpo_batch(model, n_prompts=2, n=4, prompt_len=64, response_len=96, image_grid=(1, 4, 8),
                              min_response=8, seed=seed, device=DEV)
    if not images:
        data.non_tensor_batch.pop("multi_modal_inputs")
    b = data.batch
    B, R = b["responses"].shape
    with torch.no_grad():
        m64 = copy.deepcopy(model).double()
        logits = _padded_logits(m64, data, list(range(B)), torch.float64)
        lp0 = torch.stack([ref.logprobs_from_logits(r, lab) for r, lab in zip(logits, b["responses"], strict=True)])
        lp0 = lp0.float()
        del m64, logits
    g = torch.Generator(device=DEV).manual_seed(seed)
    # old = lp0 + {-0.5, 0, +0.5}: ratios 1 (unclipped) or e^{+-0.5} (clipped), none within bf16
    # noise of the 1 +- 0.2 clip boundary, so both computations take the same clip branch per token
    # (a token near the boundary flips branch on rounding noise and its gradient jumps)
    b["old_log_probs"] = lp0 + 0.5 * torch.randint(-1, 2, (B, R), device=DEV, generator=g).float()
    b["ref_log_prob"] = lp0 + 0.1 * torch.randn(B, R, device=DEV, generator=g)
    b["advantages"] = torch.randn(B, R, device=DEV, generator=g) * b["response_mask"]
    data.meta_info.update(temperature=1.0, micro_batch_size=MB, use_dynamic_bsz=False)
    return data


def _reference(model, data, dtype):
    """dp_actor.py padded path (position ids transposed to (3, bs, S), pixel values of the
    micro-batch's rows) + the oracle loss with parameters in ``dtype``."""
    model = model.double() if dtype == torch.float64 else _params_to(model, dtype)
    model.zero_grad()
    b = data.batch
    B = b["responses"].shape[0]
    lps, pgs = [], []
    for s in range(0, B, MB):
        rows = list(range(s, s + MB))
        mb = {k: v[s : s + MB] for k, v in b.items()}
        logits = _padded_logits(model, data, rows, dtype if dtype == torch.float64 else None)
        if dtype == torch.float64:
            lp = torch.stack([ref.logprobs_from_logits(r, lab) for r, lab in zip(logits, mb["responses"], strict=True)])
            cast = torch.float64
        else:
            lp = torch.stack([ref.logprobs_fp32_math(r, lab) for r, lab in zip(logits, mb["responses"], strict=True)])
            cast = torch.float32
        loss, met = ref.actor_loss(mb["old_log_probs"].to(cast), lp, mb["advantages"].to(cast), mb["response_mask"],
                                   clip_ratio=LOSS["clip_ratio"], loss_agg_mode=LOSS["loss_agg_mode"],
                                   ref_log_prob=mb["ref_log_prob"].to(cast), kl_loss_type=LOSS["ref_kl"],
                                   kl_loss_coef=LOSS["kl_coef"], grad_scale=MB / B)
        loss.backward()
        lps.append(lp.detach().double())
        pgs.append(float(met["pg_loss"]))
    grads = {n: p.grad.detach().double().clone() for n, p in model.named_parameters() if p.grad is not None}
    return torch.cat(lps), pgs, grads


def _actor(model, fused_model_ops=True, pad_multiple=64):
    from verl_amd.utils.config import actor_config
    from verl_amd.workers.actor import DataParallelPPOActor
    from verl_amd.workers.grad_sync import MixedPrecisionParams

    mgr = MixedPrecisionParams(model, bucket_bytes=1 << 20)
    opt = torch.optim.AdamW(mgr.optimizer_params(), lr=1e-6)
    cfg = actor_config(ppo_mini_batch_size=8, ppo_micro_batch_size_per_gpu=MB, use_kl_loss=True,
                       kl_loss_coef=LOSS["kl_coef"], kl_loss_type=LOSS["ref_kl"], clip_ratio=LOSS["clip_ratio"],
                       clip_ratio_c=3.0, loss_agg_mode=LOSS["loss_agg_mode"], entropy_coeff=0,
                       use_remove_padding=True, pack_pad_multiple=pad_multiple, logprob_inplace_backward=False,
                       grad_clip=1e9, fused_model_ops=fused_model_ops)
    return DataParallelPPOActor(cfg, model, opt, grad_reducer=mgr), mgr


def _run(model, data, fused_model_ops=True):
    actor, mgr = _actor(model, fused_model_ops)
    lp, ent = actor.compute_log_prob(data, calculate_entropy=True)
    assert torch.isfinite(ent).all()
    grads = {}

    def capture():
        mgr.finish_sync()
        for (n, p), m in zip(model.named_parameters(), mgr.optimizer_params(), strict=True):
            if m.grad is not None:
                grads[n] = m.grad.detach().double().clone()
        return torch.tensor(0.0, device=DEV)

    actor._optimizer_step = capture
    metrics = actor.update_policy(data)
    assert bool(actor._fused_backbone) == fused_model_ops
    return lp.double(), metrics["actor/pg_loss"], grads


def _rel(g, g64):
    num = sum(float((g[n] - g64[n]).square().sum()) for n in g64)
    den = sum(float(g64[n].square().sum()) for n in g64)
    return (num / den) ** 0.5


@pytest.mark.parametrize("images,fused", [(True, True), (False, True), (True, False)],
                         ids=["images-fused", "mrope-text-fused", "images-hf-decoder"])
def test_qwen2_vl_actor_within_bf16_budget_of_fp64(images, fused):
    torch.manual_seed(0)
    base = _tiny_vl()
    data = _data(base, images=images)
    pos = data.batch["position_ids"]
    assert pos.shape[1] == 3 and not torch.equal(pos[:, 0], pos[:, 1])  # genuinely 3-D positions
    m = data.batch["response_mask"].bool()
    lp64, pg64, g64 = _reference(copy.deepcopy(base), data, torch.float64)
    lp16, pg16, g16 = _reference(copy.deepcopy(base), data, torch.bfloat16)
    lpb, pgb, gb = _run(copy.deepcopy(base), data, fused_model_ops=fused)
    e_ref = float((lp16 - lp64)[m].abs().max())
    e_b = float((lpb - lp64)[m].abs().max())
    assert e_b <= 2 * e_ref + 2e-3, ("log-prob", e_b, e_ref)
    for b_, r_, x in zip(pgb, pg16, pg64, strict=True):
        assert abs(b_ - x) <= 2 * abs(r_ - x) + 1e-4, ("pg_loss", b_, r_, x)
    assert set(g64) <= set(gb)
    # parameters the reference leaves without a gradient (the vision tower on text-only rows)
    # get none here either: their bucket views stay zero
    assert all(float(gb[n].abs().max()) == 0.0 for n in set(gb) - set(g64))
    gb = {n: gb[n] for n in g64}
    if images:
        assert any(n.startswith("model.visual") for n in g64)  # the vision tower trains too
    r_ref, r_b = _rel(g16, g64), _rel(gb, g64)
    assert r_b <= 2 * r_ref + 1e-3, ("grad rel err", r_b, r_ref)
    assert all(torch.isfinite(v).all() for v in gb.values())


def test_mrope_rotary_equals_hf_sections():
    """qwen2_fused.rotary's per-section row selection equals apply_multimodal_rotary_pos_emb's."""
    from transformers.models.qwen2_vl.modeling_qwen2_vl import apply_multimodal_rotary_pos_emb

    from verl_amd.workers.actor import qwen2_fused

    model = _params_to(_tiny_vl(), torch.bfloat16)
    stack = model.model.language_model
    T = 37
    pos = torch.stack([torch.arange(T), torch.arange(T) // 3, torch.arange(T) % 5]).to(DEV)
    x = torch.randn(T, 256, device=DEV, dtype=torch.bfloat16)
    cos, sin = qwen2_fused.rotary(stack, x, pos)
    c3, s3 = stack.rotary_emb(x.unsqueeze(0), pos.unsqueeze(1))
    q = torch.randn(1, 4, T, 64, device=DEV, dtype=torch.bfloat16)
    qh, _ = apply_multimodal_rotary_pos_emb(q, q, c3, s3, qwen2_fused.mrope_section(stack))
    qm = q * cos.unsqueeze(1) + torch.cat([-q[..., 32:], q[..., :32]], -1) * sin.unsqueeze(1)
    assert torch.equal(qh, qm)


def test_qwen2_vl_7b_grpo_step_one_gpu():
    """Config 4 at model size: Qwen2-VL-7B (public architecture, random init), one GRPO step with
    one image per prompt through the worker (old log-probs, GRPO advantages, update, LR
    scheduler, perf metrics) on the sharded optimizer manager."""
    import gc

    from verl_amd.trainer.ppo.trainer_step import PPOTrainerStep
    from verl_amd.utils.config import AttrDict, actor_config
    from verl_amd.utils.model import build_qwen2_vl
    from verl_amd.utils.synthetic import make_vl_grpo_batch
    from verl_amd.workers.dp_workers import ActorWorker

    gc.collect()
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats()
    n = 4
    model = build_qwen2_vl("7b", device=DEV, seed=0)
    n_text = sum(p.numel() for p in model.model.language_model.parameters()) + model.lm_head.weight.numel()
    n_vis = sum(p.numel() for p in model.model.visual.parameters())
    assert 7.0e9 < n_text < 7.8e9 and 0.5e9 < n_vis < 0.8e9, (n_text, n_vis)
    cfg = AttrDict(
        algorithm=AttrDict(adv_estimator="grpo", gamma=1.0, lam=1.0, norm_adv_by_std_in_grpo=True,
                           use_kl_in_reward=False),
        actor_rollout_ref=AttrDict(
            actor=actor_config(ppo_mini_batch_size=2, ppo_micro_batch_size_per_gpu=4, use_kl_loss=False,
                               loss_agg_mode="token-mean", grad_clip=1.0,
                               optim=AttrDict(lr=1e-6, weight_decay=0.01, warmup_style="constant",
                                              lr_warmup_steps=2)),
            rollout=AttrDict(n=n, temperature=1.0, log_prob_micro_batch_size_per_gpu=4)),
        trainer=AttrDict(critic_warmup=0, balance_batch=False))
    data = make_vl_grpo_batch(model, n_prompts=2, n=n, prompt_len=192, response_len=256, image_grid=(1, 16, 16),
                              min_response=32, seed=11)
    worker = ActorWorker(AttrDict(actor=cfg.actor_rollout_ref.actor, rollout=cfg.actor_rollout_ref.rollout),
                         rollout_n=n)
    worker.init_model(model, bucket_mb=1024, zero=True)
    before = [p.detach().clone() for p in list(model.model.language_model.parameters())[:2]]
    step = PPOTrainerStep(cfg, worker)
    out, met = step.step(data)
    assert worker.actor._fused_backbone  # the packed fused decoder ran (head_dim 128: aten flash)
    for k in ("actor/pg_loss", "actor/grad_norm", "actor/entropy", "perf/mfu/actor", "actor/lr",
              "perf/max_memory_allocated_gb"):
        assert np.isfinite(met[k]), (k, met[k])
    assert met["actor/grad_norm"] > 0 and met["actor/lr"] == 0.0  # warmup step 0 of 2
    adv = out.batch["advantages"]
    m = out.batch["response_mask"].bool()
    assert torch.isfinite(adv).all() and (adv[~m] == 0).all()
    # lr 0 on the first warmup step: AdamW's decoupled weight decay is lr-scaled too, so the
    # weights stay put; the second step (lr 5e-7) moves them
    out, met2 = step.step(data)
    assert met2["actor/lr"] == pytest.approx(5e-7)
    after = list(model.model.language_model.parameters())[:2]
    assert any(not torch.equal(a, b) for a, b in zip(after, before, strict=True))
    print("qwen2-vl 7b", {k: round(v, 5) for k, v in met2.items() if k.startswith(("actor/", "perf/"))},
          "peak GB", torch.cuda.max_memory_allocated() / 1e9)
