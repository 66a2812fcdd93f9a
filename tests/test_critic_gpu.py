"""Critic path on MI355X: the fused clipped value-loss kernel against the oracle
(core_algos.py:992-1031) including torch's tie / boundary gradients, and DataParallelPPOCritic /
CriticWorker against the reference computation on a tiny random Qwen2 value model."""

import copy

import numpy as np
import pytest
import torch

from oracle import reference_ops as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
AGGS = ["token-mean", "seq-mean-token-sum", "seq-mean-token-mean", "seq-mean-token-sum-norm"]


def _close(a, b, atol, rtol=0.0, what=""):
    a, b = a.detach().cpu().double(), b.detach().cpu().double()
    assert torch.allclose(a, b, atol=atol, rtol=rtol), f"{what}: max err {(a - b).abs().max().item():.3e}"


def _value_inputs(B, R, seed, mask_dtype=torch.int64):
    g = torch.Generator().manual_seed(seed)
    values = torch.randn(B, R, generator=g)
    vpreds = values + 0.6 * torch.randn(B, R, generator=g)  # straddles the +-0.5 clip band
    returns = values + torch.randn(B, R, generator=g)
    lens = torch.randint(1, R + 1, (B,), generator=g)
    mask = (torch.arange(R)[None, :] < lens[:, None]).to(mask_dtype)
    return vpreds, values, returns, mask


@pytest.mark.parametrize("agg", AGGS)
@pytest.mark.parametrize("mask_dtype", [torch.int64, torch.float32, torch.bool])
def test_value_loss_matches_oracle(agg, mask_dtype):
    from verl_amd import kernels as K

    vp, val, ret, mask = _value_inputs(7, 301, seed=3, mask_dtype=mask_dtype)
    vr = vp.clone().requires_grad_(True)
    loss, frac = ref.compute_value_loss(vr, ret, val, mask, 0.5, agg)
    loss.backward()
    vd = vp.to(DEV).requires_grad_(True)
    out = K.fused_value_loss(vd, val.to(DEV), ret.to(DEV), mask.to(DEV), 0.5, agg)
    out[0].backward()
    _close(out[0], loss, atol=1e-5, rtol=1e-5, what="vf_loss")
    _close(out[1], frac, atol=1e-6, what="vf_clipfrac")
    _close(out[2], ref.masked_mean(vp, mask), atol=1e-5, rtol=1e-5, what="vpred_mean")
    _close(vd.grad, vr.grad, atol=1e-7, rtol=1e-5, what="d vpreds")


def test_value_loss_ties_and_bounds_exact_grad():
    """vpreds exactly at values +- c (clamp boundaries) and l1 == l2 ties: torch.maximum /
    minimum give half the gradient to each side."""
    from verl_amd import kernels as K

    c = 0.5
    val = torch.zeros(1, 8)
    vp = torch.tensor([[0.5, -0.5, 0.25, 1.0, -1.0, 0.5, 0.0, 2.0]])
    ret = torch.tensor([[0.5, 1.0, 0.0, 0.75, -0.75, 0.25, 0.0, 0.5]])  # several l1 == l2
    mask = torch.ones(1, 8)
    vr = vp.clone().requires_grad_(True)
    loss, _ = ref.compute_value_loss(vr, ret, val, mask, c)
    loss.backward()
    vd = vp.to(DEV).requires_grad_(True)
    out = K.fused_value_loss(vd, val.to(DEV), ret.to(DEV), mask.to(DEV), c)
    out[0].backward()
    _close(vd.grad, vr.grad, atol=1e-9, rtol=1e-6, what="tie grads")


def test_value_loss_headline_size():
    """[512, 1024] (the headline shape) against the oracle, bf16 vpreds upcast exactly."""
    from verl_amd import kernels as K

    vp, val, ret, mask = _value_inputs(512, 1024, seed=8)
    vp = vp.to(torch.bfloat16)
    loss, frac = ref.compute_value_loss(vp.float(), ret, val, mask, 0.5)
    out = K.fused_value_loss(vp.to(DEV), val.to(DEV), ret.to(DEV), mask.to(DEV), 0.5).cpu()
    _close(out[0], loss, atol=1e-5, rtol=1e-5, what="vf_loss")
    _close(out[1], frac, atol=1e-6, what="vf_clipfrac")


def _batch(B=8, seed=0):
    from verl_amd.utils.synthetic import make_grpo_batch

    return make_grpo_batch(n_prompts=B // 4, n=4, prompt_len=24, response_len=40, vocab=4096, min_prompt=3,
                           dense_responses=False, min_response=5, seed=seed, device=DEV)


def _ref_values(model, b):
    R = b["responses"].shape[1]
    out = model(input_ids=b["input_ids"], attention_mask=b["attention_mask"], position_ids=b["position_ids"],
                use_cache=False).logits
    return out[:, -R - 1 : -1].squeeze(-1)


@pytest.mark.parametrize("mb,cmb", [(4, None), (4, 8), (3, 8)])
def test_critic_compute_values_and_update_match_reference(mb, cmb):
    """fp32 padded path: compute_values == HF value model slice x mask; update_critic gradients ==
    oracle clipped value loss through torch autograd on an identical model copy. cmb =
    compute_micro_batch_size_per_gpu: the loss micro-batches of mb rows aggregated one by one
    inside larger passes give the same per-micro-batch metrics and accumulated gradient."""
    from verl_amd.utils.config import critic_config
    from verl_amd.utils.model import build_qwen2_critic
    from verl_amd.workers.critic import DataParallelPPOCritic

    torch.manual_seed(0)
    model = build_qwen2_critic("tiny", device=DEV, attn_implementation="sdpa")
    model_ref = copy.deepcopy(model)
    data = _batch(seed=4)
    b = data.batch
    cfg = critic_config(ppo_mini_batch_size=8, ppo_micro_batch_size_per_gpu=mb, grad_clip=1e9, cliprange_value=0.5,
                        compute_micro_batch_size_per_gpu=cmb)
    critic = DataParallelPPOCritic(cfg, model, torch.optim.AdamW(model.parameters(), lr=1e-3))
    data.meta_info.update(micro_batch_size=3, use_dynamic_bsz=False)
    values = critic.compute_values(data)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        want = _ref_values(model_ref, b).float() * b["response_mask"]
    _close(values, want, atol=2e-2, rtol=2e-2, what="values (bf16 autocast)")

    g = torch.Generator(device=DEV).manual_seed(1)
    b["values"] = values
    b["returns"] = values + torch.randn(values.shape, device=DEV, generator=g) * b["response_mask"]
    grads = {}

    def capture():
        for n, p in model.named_parameters():
            grads[n] = p.grad.detach().clone()
        return torch.tensor(0.0, device=DEV)

    critic._optimizer_step = capture
    metrics = critic.update_critic(data)
    starts = range(0, 8, mb)
    assert len(metrics["critic/vf_loss"]) == len(starts) and len(metrics["critic/grad_norm"]) == 1
    model_ref.zero_grad()
    losses = []
    for s in starts:
        mbat = {k: v[s : s + mb] for k, v in b.items()}
        with torch.autocast("cuda", dtype=torch.bfloat16):
            vp = _ref_values(model_ref, mbat).float()
        loss, _ = ref.compute_value_loss(vp, mbat["returns"], mbat["values"], mbat["response_mask"], 0.5)
        (loss / (8 // mb)).backward()
        losses.append(loss.item())
    assert np.allclose(metrics["critic/vf_loss"], losses, atol=1e-4, rtol=1e-3)
    for n, p in model_ref.named_parameters():
        scale = p.grad.abs().max().item() + 1e-12
        err = (grads[n] - p.grad).abs().max().item()
        assert err <= 5e-2 * scale + 1e-6, (n, err, scale)


def _critic_builder(family):
    from verl_amd.utils.model import build_llama_critic, build_qwen2_critic

    return {"qwen2": build_qwen2_critic, "llama": build_llama_critic}[family]


@pytest.mark.parametrize("family", ["qwen2", "llama"])
def test_packed_critic_matches_padded(family):
    """use_remove_padding (fused packed backbone, value head on response positions only) vs the
    padded HF path: same values to bf16 level, same loss. Llama = BASELINE config 3's critic
    architecture (tiny, with Llama-3.1 rope scaling)."""
    from verl_amd.utils.config import AttrDict, critic_config
    from verl_amd.workers.actor import attention
    from verl_amd.workers.critic import DataParallelPPOCritic

    if not attention.varlen_available(DEV):
        pytest.skip("flash varlen unavailable")
    base = _critic_builder(family)("tiny", device=DEV, attn_implementation="sdpa", seed=2)
    for p in base.parameters():
        p.data = p.data.to(torch.bfloat16)
    data = _batch(seed=6)
    data.meta_info.update(micro_batch_size=4, use_dynamic_bsz=False)
    out = {}
    for rmpad in (False, True):
        m = copy.deepcopy(base)
        cfg = critic_config(ppo_mini_batch_size=8, ppo_micro_batch_size_per_gpu=4,
                            model=AttrDict(use_remove_padding=rmpad))
        c = DataParallelPPOCritic(cfg, m, torch.optim.SGD(m.parameters(), lr=0.0))
        out[rmpad] = c.compute_values(data)
        if rmpad:
            assert c._fused_backbone is True
    msk = data.batch["response_mask"].bool()
    _close(out[True][msk], out[False][msk], atol=5e-2, rtol=3e-2, what="packed vs padded values")
    assert (out[True][~msk] == 0).all()


@pytest.mark.parametrize("family,lr", [("qwen2", 2e-4), ("llama", 5e-5)])
def test_critic_worker_gae_step(family, lr):
    """CriticWorker end to end with bf16/fp32-master mixed precision and dynamic bsz: values ->
    GAE (HIP scan) -> repeated critic updates on the same targets; the value loss falls."""
    from verl_amd.trainer.ppo.core_algos import AdvantageEstimator
    from verl_amd.trainer.ppo.ray_trainer import compute_advantage
    from verl_amd.utils.config import AttrDict, critic_config
    from verl_amd.workers.actor import attention
    from verl_amd.workers.dp_workers import CriticWorker

    rmpad = attention.varlen_available(DEV)
    cfg = critic_config(ppo_mini_batch_size=8, ppo_micro_batch_size_per_gpu=None, use_dynamic_bsz=True,
                        ppo_max_token_len_per_gpu=256, forward_max_token_len_per_gpu=256,
                        model=AttrDict(use_remove_padding=rmpad), optim=AttrDict(lr=lr, weight_decay=0.0))
    w = CriticWorker(cfg).init_model(_critic_builder(family)("tiny", device=DEV, attn_implementation="sdpa", seed=5))
    data = _batch(seed=9)
    data.batch["values"] = w.compute_values(data).batch["values"]
    compute_advantage(data, AdvantageEstimator.GAE, gamma=1.0, lam=0.95)
    assert torch.isfinite(data.batch["returns"]).all()
    losses = []
    for _ in range(6):  # same targets: repeated critic updates must reduce the value loss
        met = w.update_critic(data).meta_info["metrics"]
        assert all(np.isfinite(v) for v in met["critic/vf_loss"])
        losses.append(float(np.mean(met["critic/vf_loss"])))
        assert met["critic/lr"] == lr
    assert losses[-1] < losses[0], losses


def test_critic_dynamic_bsz_merged_passes_match_reference_micro_batches():
    """use_dynamic_bsz with compute_max_token_len_per_gpu: the token-budget micro-batches merged into
    larger passes (the fused value loss aggregating each by its row offsets) give the reference's
    per-micro-batch vf_loss list and accumulated gradient (sum of vf_loss_s * rows_s / mini,
    dp_critic.py:218-232), against one pass per micro-batch on an identical model copy."""
    from verl_amd.utils.config import critic_config
    from verl_amd.utils.model import build_qwen2_critic
    from verl_amd.workers.critic import DataParallelPPOCritic

    torch.manual_seed(0)
    model = build_qwen2_critic("tiny", device=DEV, attn_implementation="sdpa")
    model_ref = copy.deepcopy(model)
    data = _batch(seed=12)
    b = data.batch
    S = b["input_ids"].shape[1]
    g = torch.Generator(device=DEV).manual_seed(3)
    b["values"] = torch.randn(b["response_mask"].shape, device=DEV, generator=g) * b["response_mask"]
    b["returns"] = b["values"] + torch.randn(b["values"].shape, device=DEV, generator=g) * b["response_mask"]
    grads, metrics = [], []
    for m, merge in ((model_ref, None), (model, 100 * S)):
        cfg = critic_config(ppo_mini_batch_size=8, ppo_micro_batch_size_per_gpu=None, use_dynamic_bsz=True,
                            ppo_max_token_len_per_gpu=2 * S, grad_clip=1e9, cliprange_value=0.5,
                            compute_max_token_len_per_gpu=merge)
        critic = DataParallelPPOCritic(cfg, m, torch.optim.AdamW(m.parameters(), lr=1e-3))
        got = {}

        def capture(m=m, got=got):
            for n, p in m.named_parameters():
                got[n] = p.grad.detach().clone()
            return torch.tensor(0.0, device=DEV)

        critic._optimizer_step = capture
        metrics.append(critic.update_critic(data))
        grads.append(got)
    ref_l, new_l = metrics[0]["critic/vf_loss"], metrics[1]["critic/vf_loss"]
    assert len(ref_l) == len(new_l) > 2
    assert np.allclose(new_l, ref_l, atol=1e-3, rtol=2e-2), (new_l, ref_l)
    for n in grads[0]:
        scale = grads[0][n].abs().max().item() + 1e-12
        err = (grads[1][n] - grads[0][n]).abs().max().item()
        assert err <= 5e-2 * scale + 1e-6, (n, err, scale)
