"""Actor-level parity on MI355X: DataParallelPPOActor vs the reference computation written with
the oracle (dp_actor.py semantics) on a tiny random Qwen2 model."""

import copy

import numpy as np
import pytest
import torch

from oracle import reference_ops as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _batch(B=8, P=24, R=40, V=4096, seed=0, dense=False):
    from verl_amd.utils.synthetic import make_grpo_batch

    return make_grpo_batch(n_prompts=B // 4, n=4, prompt_len=P, response_len=R, vocab=V, min_prompt=3,
                           dense_responses=dense, min_response=5, seed=seed, device=DEV)


def _actor(model, **cfg):
    from verl_amd.utils.config import actor_config
    from verl_amd.workers.actor import DataParallelPPOActor

    c = actor_config(**cfg)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3)
    return DataParallelPPOActor(c, model, opt)


def _ref_logprobs(model, data, temperature):
    """dp_actor.py non-rmpad path (:239-268) with the oracle's log-prob/entropy, fp32."""
    b = data.batch
    R = b["responses"].shape[1]
    logits = model(input_ids=b["input_ids"], attention_mask=b["attention_mask"], position_ids=b["position_ids"],
                   use_cache=False).logits
    logits = logits.div(temperature)[:, -R - 1 : -1, :]
    lp = torch.stack([ref.logprobs_from_logits(row, lab) for row, lab in zip(logits, b["responses"], strict=True)])
    ent = ref.entropy_from_logits(logits)
    return lp, ent


@pytest.mark.parametrize("temperature", [1.0, 0.8])
def test_compute_log_prob_fp32_matches_reference(temperature):
    from verl_amd.utils.model import build_qwen2

    model = build_qwen2("tiny", device=DEV, attn_implementation="sdpa")
    data = _batch()
    actor = _actor(model, use_remove_padding=False, autocast_dtype=None)
    data.meta_info.update(micro_batch_size=3, temperature=temperature, use_dynamic_bsz=False)
    lp, ent = actor.compute_log_prob(data, calculate_entropy=True)
    with torch.no_grad():
        want_lp, want_ent = _ref_logprobs(model, data, temperature)
    m = data.batch["response_mask"].bool()
    assert torch.allclose(lp[m], want_lp[m], atol=1e-4, rtol=1e-4)
    assert torch.allclose(ent[m], want_ent[m], atol=1e-4, rtol=1e-4)


def test_rmpad_varlen_path_matches_padded_path():
    from verl_amd.utils.model import build_qwen2
    from verl_amd.workers.actor import attention

    if not attention.varlen_available(DEV):
        pytest.skip("PyTorch-ROCm flash varlen attention unavailable on this device")
    model = build_qwen2("tiny", device=DEV, attn_implementation="sdpa")
    data = _batch(seed=3)
    data.meta_info.update(micro_batch_size=4, temperature=1.0, use_dynamic_bsz=False)
    padded = _actor(model, use_remove_padding=False)
    lp_pad, ent_pad = padded.compute_log_prob(data, calculate_entropy=True)
    model2 = copy.deepcopy(model)
    packed = _actor(model2, use_remove_padding=True)
    lp_pk, ent_pk = packed.compute_log_prob(data, calculate_entropy=True)
    m = data.batch["response_mask"].bool()
    # both bf16 autocast; different attention kernels -> bf16-level agreement
    assert torch.allclose(lp_pk[m], lp_pad[m], atol=5e-2, rtol=2e-2), (lp_pk[m] - lp_pad[m]).abs().max()
    assert torch.allclose(ent_pk[m], ent_pad[m], atol=5e-2, rtol=2e-2)
    # masked positions as the reference's rmpad path fills them (dp_actor.py:131-137, 219-237): the
    # last real token of a short row scores the rolled packed stream's next token (the next row's
    # first real token in the micro-batch of 4, wrapping), later positions are pad_input zeros
    with torch.no_grad():
        want_lp, want_ent = _ref_rmpad_masked(model, data, 1.0, micro=4)
    assert torch.allclose(lp_pk, want_lp, atol=5e-2, rtol=2e-2), (lp_pk - want_lp).abs().max()
    assert torch.allclose(ent_pk, want_ent, atol=5e-2, rtol=2e-2), (ent_pk - want_ent).abs().max()
    tail = (~m) & (want_lp != 0)
    assert tail.any() and (lp_pk[tail] != 0).all()


def _ref_rmpad_masked(model, data, temperature, micro):
    """The reference's remove-padding log-probs / entropies at EVERY response position
    (dp_actor.py:99-237): labels = torch.roll(input_ids_rmpad, -1) within each micro-batch of
    ``micro`` rows, pad_input zeros at padding; logits from the padded forward (same values at real
    positions up to attention-kernel rounding), fp32 oracle log-softmax / entropy."""
    b = data.batch
    ids, am = b["input_ids"], b["attention_mask"].bool()
    B, S = ids.shape
    R = b["responses"].shape[1]
    logits = model(input_ids=ids, attention_mask=b["attention_mask"], position_ids=b["position_ids"],
                   use_cache=False).logits.float().div(temperature)
    lp = torch.zeros(B, R, device=ids.device)
    ent = torch.zeros(B, R, device=ids.device)
    first = am.long().argmax(dim=1)
    for r in range(B):
        g0 = r // micro * micro
        g1 = min(g0 + micro, B)
        for t in range(R):
            p = S - R - 1 + t
            if not am[r, p]:
                continue
            if am[r, p + 1]:
                lab = ids[r, p + 1]
            else:
                nr = r + 1 if r + 1 < g1 else g0
                lab = ids[nr, first[nr]]
            lp[r, t] = ref.logprobs_from_logits(logits[r, p][None], lab[None])[0]
            ent[r, t] = ref.entropy_from_logits(logits[r, p][None])[0]
    return lp, ent


@pytest.mark.parametrize("agg,mb,cmb", [("token-mean", 4, None), ("seq-mean-token-mean", 4, None),
                                         ("token-mean", 4, 8), ("seq-mean-token-mean", 3, 6),
                                         ("seq-mean-token-sum", 2, 8), ("seq-mean-token-sum-norm", 3, 8)])
def test_update_policy_gradients_match_reference(agg, mb, cmb):
    """One mini-batch of update_policy (fp32, padded path) vs the reference loss written with
    the oracle and torch autograd on an identical model copy: same gradients, same metrics.
    cmb = compute_micro_batch_size_per_gpu: several loss micro-batches of mb rows in one pass
    (the fused loss aggregates each on its own) must give the reference's per-micro-batch
    metric lists and its accumulated gradient (micro-batches [0:mb], [mb:2mb], ..., the last
    one ragged when mb does not divide 8)."""
    from verl_amd.utils.model import build_qwen2

    torch.manual_seed(0)
    model = build_qwen2("tiny", device=DEV, attn_implementation="sdpa")
    model_ref = copy.deepcopy(model)
    data = _batch(B=8, seed=5)
    b = data.batch
    R = b["responses"].shape[1]
    with torch.no_grad():
        lp0, _ = _ref_logprobs(model_ref, data, 1.0)
    g = torch.Generator(device=DEV).manual_seed(1)
    b["old_log_probs"] = lp0 + 0.05 * torch.randn(lp0.shape, device=DEV, generator=g)
    b["ref_log_prob"] = lp0 + 0.1 * torch.randn(lp0.shape, device=DEV, generator=g)
    b["advantages"] = torch.randn(8, R, device=DEV, generator=g) * b["response_mask"]
    data.meta_info.update(temperature=1.0)
    cfg = dict(use_remove_padding=False, autocast_dtype=None, ppo_mini_batch_size=8, ppo_micro_batch_size_per_gpu=mb,
               use_kl_loss=True, kl_loss_type="low_var_kl", kl_loss_coef=0.01, loss_agg_mode=agg, entropy_coeff=0.01,
               clip_ratio=0.2, grad_clip=1e9, compute_micro_batch_size_per_gpu=cmb)
    actor = _actor(model, **cfg)
    # capture gradients before the optimizer step
    grads = {}

    def capture():
        for n, p in model.named_parameters():
            grads[n] = p.grad.detach().clone()
        return torch.tensor(0.0, device=DEV)

    actor._optimizer_step = capture
    metrics = actor.update_policy(data)
    if cmb:
        assert actor._pass_rows("vanilla") == cmb // mb * mb
    # reference: the same micro-batches of mb rows, oracle loss, torch autograd, / (8 // mb)
    model_ref.zero_grad()
    pg_losses, kl_losses = [], []
    for s in range(0, 8, mb):
        sl = slice(s, s + mb)
        mbat = {k: v[sl] for k, v in b.items()}
        out = model_ref(input_ids=mbat["input_ids"], attention_mask=mbat["attention_mask"],
                        position_ids=mbat["position_ids"], use_cache=False).logits[:, -R - 1 : -1, :]
        lp = torch.stack([ref.logprobs_from_logits(r, lab) for r, lab in zip(out, mbat["responses"], strict=True)])
        ent = ref.entropy_from_logits(out)
        loss, met = ref.actor_loss(mbat["old_log_probs"], lp, mbat["advantages"], mbat["response_mask"], clip_ratio=0.2,
                                   loss_agg_mode=agg, entropy=ent, entropy_coeff=0.01, ref_log_prob=mbat["ref_log_prob"],
                                   kl_loss_type="low_var_kl", kl_loss_coef=0.01, grad_scale=1.0 / (8 // mb))
        loss.backward()
        pg_losses.append(met["pg_loss"].item())
        kl_losses.append(met["kl_loss"].item())
    assert len(metrics["actor/pg_loss"]) == len(pg_losses) == len(metrics["actor/kl_coef"])
    assert np.allclose(metrics["actor/pg_loss"], pg_losses, atol=1e-5, rtol=1e-4)
    assert np.allclose(metrics["actor/kl_loss"], kl_losses, atol=1e-6, rtol=1e-4)
    for n, p in model_ref.named_parameters():
        gr = p.grad
        scale = gr.abs().max().item() + 1e-12
        assert torch.allclose(grads[n], gr, atol=1e-4 * scale, rtol=1e-3), (n, (grads[n] - gr).abs().max().item(), scale)


def test_worker_step_runs_and_learns():
    """ActorWorker end to end on the tiny model: old-logp, GRPO advantages, one update."""
    from verl_amd.trainer.ppo.core_algos import AdvantageEstimator
    from verl_amd.trainer.ppo.ray_trainer import compute_advantage
    from verl_amd.utils.config import AttrDict, actor_config
    from verl_amd.utils.model import build_qwen2
    from verl_amd.workers.actor import attention
    from verl_amd.workers.dp_workers import ActorWorker

    rmpad = attention.varlen_available(DEV)
    cfg = AttrDict(actor=actor_config(ppo_mini_batch_size=2, ppo_micro_batch_size_per_gpu=4, use_kl_loss=True,
                                      use_remove_padding=rmpad),
                   rollout=AttrDict(log_prob_micro_batch_size_per_gpu=8, temperature=1.0))
    w = ActorWorker(cfg, rollout_n=4).init_model(build_qwen2("tiny", device=DEV, attn_implementation="sdpa"))
    data = _batch(B=8, seed=9)
    out = w.compute_log_prob(data)
    data.batch["old_log_probs"] = out.batch["old_log_probs"]
    data.batch["ref_log_prob"] = out.batch["old_log_probs"].clone()
    compute_advantage(data, AdvantageEstimator.GRPO)
    res = w.update_actor(data)
    met = res.meta_info["metrics"]
    assert len(met["actor/pg_loss"]) == 2 and len(met["actor/grad_norm"]) == 1
    assert all(np.isfinite(v) for v in met["actor/pg_loss"])
    # first update: lp == old -> ratio 1, no clipping, kl 0
    assert max(met["actor/pg_clipfrac"]) == 0.0
    assert abs(met["actor/ppo_kl"][0]) < 1e-3


@pytest.mark.parametrize("merge", [None, 3, 100])
def test_dynamic_bsz_log_prob_and_update_match_reference(merge):
    """use_dynamic_bsz (dp_actor.py:321-347, 382-384, 465-467): token-budget micro-batches give the
    same log-probs as fixed micro-batches, and update_policy's gradient is the reference's sum of
    per-micro-batch losses scaled by rows / ppo_mini_batch_size. merge: compute_max_token_len_per_gpu
    = merge x the micro-batch budget, so passes hold several micro-batches (aggregated one by one
    from their row offsets: same metric lists, same gradient)."""
    from verl_amd.utils.model import build_qwen2
    from verl_amd.utils.seqlen_balancing import prepare_dynamic_batch

    torch.manual_seed(0)
    model = build_qwen2("tiny", device=DEV, attn_implementation="sdpa")
    model_ref = copy.deepcopy(model)
    data = _batch(B=8, seed=6)
    b = data.batch
    R = b["responses"].shape[1]
    S = b["input_ids"].shape[1]
    budget = 2 * S  # several micro-batches of uneven row counts
    actor = _actor(model, use_remove_padding=False, autocast_dtype=None, ppo_mini_batch_size=8,
                   ppo_micro_batch_size_per_gpu=None, use_dynamic_bsz=True, ppo_max_token_len_per_gpu=budget,
                   use_kl_loss=False, entropy_coeff=0.0, clip_ratio=0.2, grad_clip=1e9,
                   compute_max_token_len_per_gpu=merge * budget if merge else None)
    data.meta_info.update(micro_batch_size=None, temperature=1.0, use_dynamic_bsz=True, max_token_len=budget)
    lp_dyn, ent_dyn = actor.compute_log_prob(data, calculate_entropy=True)
    with torch.no_grad():
        want_lp, want_ent = _ref_logprobs(model_ref, data, 1.0)
    m = b["response_mask"].bool()
    assert torch.allclose(lp_dyn[m], want_lp[m], atol=1e-4, rtol=1e-4)
    assert torch.allclose(ent_dyn[m], want_ent[m], atol=1e-4, rtol=1e-4)

    g = torch.Generator(device=DEV).manual_seed(2)
    b["old_log_probs"] = want_lp + 0.05 * torch.randn(want_lp.shape, device=DEV, generator=g)
    b["advantages"] = torch.randn(8, R, device=DEV, generator=g) * b["response_mask"]
    grads = {}

    def capture():
        for n, p in model.named_parameters():
            grads[n] = p.grad.detach().clone()
        return torch.tensor(0.0, device=DEV)

    actor._optimizer_step = capture
    metrics = actor.update_policy(data)
    sel = data.select(batch_keys=["responses", "response_mask", "input_ids", "attention_mask", "position_ids",
                                  "old_log_probs", "advantages"])
    micro, idx_lists = prepare_dynamic_batch(sel, max_token_len=budget)
    assert len(micro) > 2 and len({len(ix) for ix in idx_lists}) >= 1
    model_ref.zero_grad()
    pg_losses = []
    for mbp in micro:
        mb = mbp.batch
        out = model_ref(input_ids=mb["input_ids"], attention_mask=mb["attention_mask"],
                        position_ids=mb["position_ids"], use_cache=False).logits[:, -R - 1 : -1, :]
        lp = torch.stack([ref.logprobs_from_logits(r, lab) for r, lab in zip(out, mb["responses"], strict=True)])
        loss, met = ref.actor_loss(mb["old_log_probs"], lp, mb["advantages"], mb["response_mask"], clip_ratio=0.2,
                                   loss_agg_mode="token-mean", grad_scale=len(mbp) / 8)
        loss.backward()
        pg_losses.append(met["pg_loss"].item())
    assert np.allclose(metrics["actor/pg_loss"], pg_losses, atol=1e-5, rtol=1e-4)
    for n, p in model_ref.named_parameters():
        scale = p.grad.abs().max().item() + 1e-12
        assert torch.allclose(grads[n], p.grad, atol=1e-4 * scale, rtol=1e-3), n


@pytest.mark.parametrize("pad", [64, 1000])
def test_pack_pad_multiple_leaves_results_unchanged(pad):
    """pack_pad_multiple appends one dummy sequence to every packed micro-batch (fixed GEMM
    shapes for the tuned table): log-probs, entropies and the weight gradients of the real tokens
    must match the unpadded run on the fused bf16 backbone."""
    from verl_amd.utils.model import build_qwen2

    torch.manual_seed(0)
    model = build_qwen2("tiny", device=DEV, dtype=torch.bfloat16)
    model2 = copy.deepcopy(model)
    data = _batch(B=8, seed=11)
    b = data.batch
    R = b["responses"].shape[1]
    data.meta_info.update(micro_batch_size=4, temperature=1.0, use_dynamic_bsz=False)
    cfg = dict(ppo_mini_batch_size=8, ppo_micro_batch_size_per_gpu=4, use_kl_loss=False, grad_clip=1e9)
    a0 = _actor(model, **cfg)
    a1 = _actor(model2, pack_pad_multiple=pad, **cfg)
    lp0, ent0 = a0.compute_log_prob(data, calculate_entropy=True)
    lp1, ent1 = a1.compute_log_prob(data, calculate_entropy=True)
    m = b["response_mask"].bool()
    assert torch.allclose(lp1[m], lp0[m], atol=1e-2, rtol=1e-2), (lp1[m] - lp0[m]).abs().max()
    assert torch.allclose(ent1[m], ent0[m], atol=1e-2, rtol=1e-2)
    g = torch.Generator(device=DEV).manual_seed(2)
    b["old_log_probs"] = lp0 + 0.05 * torch.randn(lp0.shape, device=DEV, generator=g)
    b["advantages"] = torch.randn(8, R, device=DEV, generator=g) * b["response_mask"]
    grads = [{}, {}]
    for i, (a, mdl) in enumerate(((a0, model), (a1, model2))):
        def capture(mdl=mdl, i=i):
            for n, p in mdl.named_parameters():
                grads[i][n] = p.grad.detach().float().clone()
            return torch.tensor(0.0, device=DEV)

        a._optimizer_step = capture
        a.update_policy(data)
    for n in grads[0]:
        g0, g1 = grads[0][n], grads[1][n]
        scale = g0.abs().max().item() + 1e-12
        assert torch.allclose(g1, g0, atol=2e-2 * scale, rtol=2e-2), (n, (g1 - g0).abs().max().item(), scale)
