"""GPU parity of the gfx950 kernels against the CPU oracle (oracle/reference_ops.py).

Tolerances: the north star's 1e-4 for fp32 outputs (abs + rel); gradients written in bf16
are compared at bf16 resolution (2^-8 relative), as the reference's own kernel tests do
(tests/utils/test_linear_cross_entropy.py:260-275 use 2e-2 / 4e-2 for kernel grads).
"""

import numpy as np
import pytest
import torch

from oracle import reference_ops as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(a, b, atol=1e-4, rtol=1e-4, what=""):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    assert a.shape == b.shape, (what, a.shape, b.shape)
    nan_a, nan_b = torch.isnan(a), torch.isnan(b)
    assert torch.equal(nan_a, nan_b), f"{what}: NaN pattern differs"
    d = (a - b).abs()[~nan_a]
    tol = (atol + rtol * b.abs())[~nan_a]
    bad = d > tol
    assert not bad.any(), f"{what}: max abs err {d.max().item():.3e}, {int(bad.sum())} elements out of tol"


@pytest.fixture(scope="module")
def K():
    from verl_amd import kernels

    return kernels


# ------------------------------------------------------------------------------ log-prob / entropy
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32, torch.float16])
@pytest.mark.parametrize("V", [32000, 151936, 1000, 37])
@pytest.mark.parametrize("temperature", [1.0, 0.7])
def test_logprob_entropy_fwd(K, dtype, V, temperature):
    torch.manual_seed(V + int(temperature * 10))
    n = 24 if V > 100000 else 40
    logits = (torch.randn(n, V) * 2.0).to(dtype)
    labels = torch.randint(0, V, (n,))
    labels[3] = -100
    scaled = ref.apply_temperature(logits, temperature)
    want_lp = ref.logprobs_fp32_math(scaled, labels.clamp(min=0))
    want_lp[3] = 0.0
    want_h = ref.entropy_from_logits(scaled.float())
    lp, h = K.logprob_entropy(logits.to(DEV), labels.to(DEV), temperature)
    _close(lp, want_lp, what=f"logp {dtype} V={V}")
    _close(h, want_h, what=f"entropy {dtype} V={V}")


def test_logprob_row_stride_and_3d(K):
    torch.manual_seed(0)
    V = 5003
    big = torch.randn(2, 7, V + 13, dtype=torch.bfloat16)
    logits = big[..., :V]  # non-contiguous rows (stride V+13, not 16B aligned)
    labels = torch.randint(0, V, (2, 7))
    want = ref.logprobs_fp32_math(logits.reshape(-1, V), labels.reshape(-1)).view(2, 7)
    lp, h = K.logprob_entropy(logits.to(DEV), labels.to(DEV))
    _close(lp, want, what="strided logp")
    _close(h, ref.entropy_from_logits(logits.float()), what="strided entropy")


def test_logprob_bad_label_is_nan(K):
    logits = torch.randn(4, 100, device=DEV)
    labels = torch.tensor([0, 100, -5, 99], device=DEV)
    lp, _ = K.logprob_entropy(logits, labels)
    lp = lp.cpu()
    assert torch.isfinite(lp[0]) and torch.isfinite(lp[3])
    assert torch.isnan(lp[1]) and torch.isnan(lp[2])


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("temperature", [1.0, 0.6])
@pytest.mark.parametrize("with_entropy_grad", [False, True])
def test_logprob_entropy_bwd(K, dtype, temperature, with_entropy_grad):
    torch.manual_seed(7)
    n, V = 16, 32000
    base = (torch.randn(n, V) * 2.0).to(dtype)
    labels = torch.randint(0, V, (n,))
    g_lp = torch.randn(n)
    g_h = torch.randn(n) if with_entropy_grad else None
    # oracle gradient: autograd through the fp32 restatement of div_(T) -> logp / entropy
    x = base.double().requires_grad_(True)
    # value: the reference's in-dtype div_ (bf16 rounding); gradient: d(x/T)/dx = 1/T
    z_val = ref.apply_temperature(base, temperature).double()
    z = z_val + (x / temperature - (x / temperature).detach())
    lp_ref = ref.logprobs_from_logits(z, labels)
    loss = (lp_ref * g_lp.double()).sum()
    if g_h is not None:
        loss = loss + (ref.entropy_from_logits(z) * g_h.double()).sum()
    loss.backward()
    want = x.grad
    xd = base.to(DEV).requires_grad_(True)
    lp, h = K.logprob_entropy(xd, labels.to(DEV), temperature)
    out = (lp * g_lp.to(DEV)).sum()
    if g_h is not None:
        out = out + (h * g_h.to(DEV)).sum()
    out.backward()
    got = xd.grad.double().cpu()
    scale = want.abs().max().item()
    if dtype == torch.float32:
        _close(got, want, atol=1e-6 * max(scale, 1.0), rtol=1e-4, what="dlogits fp32")
    else:
        _close(got, want, atol=2e-3 * scale, rtol=1e-2, what="dlogits bf16")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n,V", [(1, 151936), (7, 151936), (5, 8200), (9, 8192), (3, 32000), (2, 4100)])
@pytest.mark.parametrize("temperature,ent_grad", [(1.0, False), (0.7, True)])
def test_logprob_bwd_flat_matches_per_row(K, dtype, n, V, temperature, ent_grad):
    """The flat-stream backward (equal chunks over the whole dense tensor) and the per-row-chunk
    backward compute each element identically: bitwise equal dlogits, including ignore_index
    (-100) and out-of-range labels, the label sitting in a chunk that straddles two rows, and V
    too narrow for the flat path (falls back)."""
    from verl_amd import _lib as L

    torch.manual_seed(n * 7 + V)
    base = (torch.randn(n, V) * 2.0).to(dtype).to(DEV)
    labels = torch.randint(0, V, (n,))
    if n > 2:
        labels[1] = -100
        labels[2] = V + 5
    labels[0] = V - 1
    labels = labels.to(DEV)
    g_lp = torch.randn(n, device=DEV)
    g_h = torch.randn(n, device=DEV) if ent_grad else None
    grads = []
    try:
        for flat in (-1, 0):
            L.call("va_set_tuning", L.VA_TUNE_BWD_FLAT, flat)
            x = base.clone().requires_grad_(True)
            lp, h = K.logprob_entropy(x, labels, temperature)
            out = (torch.nan_to_num(lp) * g_lp).sum()
            if g_h is not None:
                out = out + (h * g_h).sum()
            out.backward()
            grads.append(x.grad)
    finally:
        L.call("va_set_tuning", L.VA_TUNE_BWD_FLAT, -1)
    assert torch.equal(torch.isnan(grads[0]), torch.isnan(grads[1]))
    assert torch.equal(torch.nan_to_num(grads[0]), torch.nan_to_num(grads[1]))


def test_logprob_inplace_backward(K):
    torch.manual_seed(3)
    n, V = 8, 4096
    base = torch.randn(n, V, dtype=torch.bfloat16, device=DEV)
    labels = torch.randint(0, V, (n,), device=DEV)
    g = torch.randn(n, device=DEV)
    a = base.clone().requires_grad_(True)
    lp, _ = K.logprob_entropy(a, labels, 1.0, inplace_backward=False)
    (lp * g).sum().backward()
    leaf = base.clone().requires_grad_(True)
    logits = leaf * 1.0  # non-leaf buffer that the in-place backward may overwrite
    lp2, _ = K.logprob_entropy(logits, labels, 1.0, inplace_backward=True)
    (lp2 * g).sum().backward()
    assert torch.equal(a.grad, leaf.grad)


def test_logprob_auto_backward_falls_back_in_place_when_hbm_is_full(K):
    """"auto" writes dlogits into a fresh buffer when the allocator can provide
    it and over the logits (the reference's inplace_backward) when it cannot — here forced by
    reserving all but ~1 GiB of HBM around a 2.4 GB logits tensor. Both give bitwise the in-place
    result."""
    from verl_amd import custom_ops

    torch.manual_seed(4)
    n, V = 8192, 151936  # 2.49 GB of bf16 logits
    base = torch.randn(n, V, dtype=torch.bfloat16, device=DEV)
    labels = torch.randint(0, V, (n,), device=DEV)
    g = torch.randn(n, device=DEV)

    def run(mode):
        # logits: a non-leaf [n, V] buffer; the gradient w.r.t. it is what the backward writes (in
        # place: the logits storage itself), with no further [n, V] allocation on the way
        scale = torch.ones((), device=DEV, requires_grad=True)
        logits = base * scale
        lp, ent = K.logprob_entropy(logits, labels, 1.0, inplace_backward=mode)
        (dl,) = torch.autograd.grad((lp * g + 0.1 * ent).sum(), logits)
        return dl

    want = run(True)
    f0 = custom_ops.AUTO_INPLACE_FALLBACKS
    assert torch.equal(run("auto"), want)  # room for the buffer: out of place
    assert custom_ops.AUTO_INPLACE_FALLBACKS == f0
    # leave ~1 GiB beyond the logits of the next run: the 2.49 GB dlogits buffer cannot be allocated
    torch.cuda.empty_cache()
    free, _ = torch.cuda.mem_get_info()
    hog = torch.empty(max(0, free - base.numel() * base.element_size() - (1 << 30)), dtype=torch.uint8, device=DEV)
    try:
        got = run("auto")
    finally:
        del hog
        torch.cuda.empty_cache()
    assert custom_ops.AUTO_INPLACE_FALLBACKS == f0 + 1
    assert torch.equal(got, want)
    with pytest.raises(ValueError, match="auto"):
        K.logprob_entropy(base, labels, 1.0, inplace_backward="sometimes")


# ------------------------------------------------------------------------------ policy loss
def _policy_inputs(B, R, seed, mask_dtype=torch.int64, ties=True):
    g = torch.Generator().manual_seed(seed)
    new = -torch.rand(B, R, generator=g) * 3
    old = new + torch.randn(B, R, generator=g) * 0.3
    adv = torch.randn(B, R, generator=g)
    ref_lp = new + torch.randn(B, R, generator=g) * 0.1
    ent = torch.rand(B, R, generator=g) * 5
    lens = torch.randint(1, R + 1, (B,), generator=g)
    mask = (torch.arange(R)[None, :] < lens[:, None]).to(mask_dtype)
    if ties:
        # exact boundary / tie cases: ratio == 1, ratio at the clip bounds, advantage 0,
        # large |delta| beyond the +-20 clamp, and the dual-clip tie
        old[0, :4] = new[0, :4]
        adv[0, 4] = 0.0
        old[0, 5] = new[0, 5] + 25.0
        old[0, 6] = new[0, 6] - 25.0
        # r = exp(lp-old) == 1.2f / 0.8f happen only approximately; force via log
        new[0, 7] = old[0, 7] + float(np.log(np.float32(1.2)))
        new[0, 8] = old[0, 8] + float(np.log(np.float32(0.8)))
        adv[0, 9] = -1.0
        new[0, 9] = old[0, 9] + float(np.log(3.0))
    return old, new, adv, mask, ref_lp, ent


@pytest.mark.parametrize("agg", ["token-mean", "seq-mean-token-sum", "seq-mean-token-mean", "seq-mean-token-sum-norm"])
@pytest.mark.parametrize("kl", [None, "low_var_kl", "kl", "abs", "mse"])
@pytest.mark.parametrize("mask_dtype", [torch.int64, torch.float32, torch.bool])
def test_fused_policy_loss(K, agg, kl, mask_dtype):
    B, R = 8, 300
    old, new, adv, mask, ref_lp, ent = _policy_inputs(B, R, seed=11, mask_dtype=mask_dtype)
    ent_coeff, kl_coef, scale = 0.01, 0.001, 0.25
    # oracle (fp32 on CPU) with autograd
    newr = new.clone().requires_grad_(True)
    entr = ent.clone().requires_grad_(True)
    loss_ref, met = ref.actor_loss(
        old, newr, adv, mask, clip_ratio=0.2, clip_ratio_low=0.2, clip_ratio_high=0.28, clip_ratio_c=3.0,
        loss_agg_mode=agg, entropy=entr, entropy_coeff=ent_coeff,
        ref_log_prob=ref_lp if kl else None, kl_loss_type=kl or "low_var_kl", kl_loss_coef=kl_coef,
        grad_scale=scale,
    )
    loss_ref.backward()
    # kernel
    newd = new.to(DEV).requires_grad_(True)
    entd = ent.to(DEV).requires_grad_(True)
    out = K.fused_policy_loss(
        old.to(DEV), newd, adv.to(DEV), mask.to(DEV), 0.2, 0.28, 3.0, agg,
        ref_log_prob=ref_lp.to(DEV) if kl else None, kl_loss_type=kl, entropy=entd,
    )
    loss = out[0] - out[5] * ent_coeff
    if kl:
        loss = loss + out[4] * kl_coef
    (loss * scale).backward()
    _close(out[0], met["pg_loss"], what="pg_loss")
    _close(out[1], met["pg_clipfrac"], what="clipfrac")
    _close(out[2], met["ppo_kl"], what="ppo_kl")
    _close(out[3], met["pg_clipfrac_lower"], what="clipfrac_lower")
    _close(out[5], ref.agg_loss(ent, mask, agg), what="entropy_loss")
    if kl:
        _close(out[4], met["kl_loss"], what="kl_loss")
    gmax = newr.grad.abs().max().item()
    _close(newd.grad, newr.grad, atol=1e-6 * gmax + 1e-12, rtol=1e-4, what="d log_prob")
    _close(entd.grad, entr.grad, atol=1e-9, rtol=1e-4, what="d entropy")


def test_policy_loss_boundaries_exact_grad(K):
    """Tie / clamp-boundary gradients follow torch autograd (maximum/minimum 1/2 split)."""
    B, R = 1, 16
    old, new, adv, mask, _, _ = _policy_inputs(B, R, seed=5, mask_dtype=torch.float32)
    mask[:] = 1
    newr = new.clone().requires_grad_(True)
    pg, *_ = ref.compute_policy_loss(old, newr, adv, mask, cliprange=0.2, clip_ratio_c=3.0)
    pg.backward()
    newd = new.to(DEV).requires_grad_(True)
    out = K.fused_policy_loss(old.to(DEV), newd, adv.to(DEV), mask.to(DEV), 0.2, 0.2, 3.0)
    out[0].backward()
    _close(newd.grad, newr.grad, atol=1e-9, rtol=1e-5, what="boundary grads")


def test_policy_loss_identity_kat(K):
    """Hand-derived KAT: lp == old -> ratio 1, clipfrac 0, pg_loss = -masked_mean(A)."""
    B, R = 4, 64
    adv = torch.randn(B, R)
    lp = torch.randn(B, R)
    mask = torch.ones(B, R, dtype=torch.int64)
    out = K.fused_policy_loss(lp.to(DEV), lp.to(DEV), adv.to(DEV), mask.to(DEV), 0.2, 0.2, 3.0).cpu()
    assert out[1].item() == 0.0 and out[2].item() == 0.0
    _close(out[0], -adv.mean(), atol=1e-6, what="-mean(A)")


# ------------------------------------------------------------------------------ kl / agg
@pytest.mark.parametrize("kl", ["kl", "k1", "abs", "mse", "k2", "low_var_kl", "k3"])
def test_kl_penalty(K, kl):
    torch.manual_seed(2)
    lp = torch.randn(513) * 5
    rf = torch.randn(513) * 5
    rf[:3] = lp[:3]
    rf[3] = lp[3] + 30  # beyond the +-20 clamp
    a = lp.clone().requires_grad_(True)
    want = ref.kl_penalty(a, rf, kl)
    g = torch.randn(513)
    (want * g).sum().backward()
    ad = lp.to(DEV).requires_grad_(True)
    got = K.kl_penalty(ad, rf.to(DEV), kl)
    (got * g.to(DEV)).sum().backward()
    _close(got, want, atol=1e-6, rtol=1e-5, what=f"kl {kl}")
    _close(ad.grad, a.grad, atol=1e-6, rtol=1e-5, what=f"dkl {kl}")


@pytest.mark.parametrize("mode", [0, 1, 2, 3, 4, 5])
def test_masked_aggregate(K, mode):
    torch.manual_seed(9)
    x = torch.randn(6, 77)
    mask = (torch.rand(6, 77) > 0.3).to(torch.int64)
    x[0, mask[0] == 0] = float("nan")  # NaN outside the mask is ignored by the where-form
    names = {0: "token-mean", 1: "seq-mean-token-sum", 2: "seq-mean-token-mean", 3: "seq-mean-token-sum-norm"}
    xr = x.clone().requires_grad_(True)
    if mode in names:
        want = ref.agg_loss(xr, mask, names[mode])
    elif mode == 4:
        want = ref.masked_sum(xr, mask)
    else:
        want = ref.masked_mean(xr, mask, axis=-1)
    g = torch.randn(want.shape)
    (want * g).sum().backward()
    xd = x.to(DEV).requires_grad_(True)
    got = K.masked_aggregate(xd, mask.to(DEV), mode)
    (got * g.to(DEV)).sum().backward()
    _close(got, want, what=f"agg mode {mode}")
    gd, gr = xd.grad.cpu(), xr.grad
    fin = torch.isfinite(gr)
    _close(gd[fin], gr[fin], atol=1e-7, rtol=1e-5, what=f"dagg mode {mode}")


# ------------------------------------------------------------------------------ advantages
@pytest.mark.parametrize("norm", [True, False])
def test_grpo_matches_oracle(K, norm):
    torch.manual_seed(4)
    B, R = 64, 200
    index = np.array([f"uid-{i // 8}" for i in range(B)], dtype=object)
    perm = np.random.RandomState(0).permutation(B)  # _balance_batch breaks contiguity
    index = index[perm]
    index[5] = "singleton"
    rewards = torch.zeros(B, R)
    lens = torch.randint(1, R + 1, (B,))
    rewards[torch.arange(B), lens - 1] = torch.randint(0, 2, (B,)).float()
    rewards[:, 0] += torch.randn(B) * 0.1  # a non-zero reward outside the mask too
    mask = (torch.arange(R)[None, :] < lens[:, None]).to(torch.int64)
    want, _ = ref.compute_grpo_outcome_advantage(rewards.clone(), mask, index, 1e-6, norm)
    from verl_amd import _lib as L

    est = L.VA_ADV_GRPO if norm else L.VA_ADV_GRPO_NOSTD
    got = K.outcome_advantage(rewards.to(DEV), mask.to(DEV), index, 1e-6, est)
    _close(got, want, atol=1e-5, rtol=1e-5, what="grpo")


def test_grpo_kat_from_reference_test(K):
    """tests/trainer/config/test_algo_config_on_cpu.py:190-192 input; hand-derived answer."""
    rewards = torch.tensor([[1.0, 0.5, 0.0], [2.0, 1.0, 0.0], [0.5, 0.2, 0.0], [1.5, 0.8, 0.0]])
    mask = torch.ones(4, 3)
    index = np.array([0, 0, 1, 1])
    from verl_amd import _lib as L

    got = K.outcome_advantage(rewards.to(DEV), mask.to(DEV), index, 1e-6, L.VA_ADV_GRPO).cpu()
    s = np.array([1.5, 3.0, 0.7, 2.3])
    exp = []
    for a, b in [(s[0], s[1]), (s[2], s[3])]:
        sd = abs(a - b) / np.sqrt(2)
        exp += [(a - (a + b) / 2) / (sd + 1e-6), (b - (a + b) / 2) / (sd + 1e-6)]
    want = torch.tensor(exp, dtype=torch.float32)[:, None].expand(4, 3)
    _close(got, want, atol=1e-6, rtol=1e-6, what="grpo KAT")


def test_rloo_matches_oracle(K):
    torch.manual_seed(8)
    B, R = 40, 50
    index = np.array([i % 7 for i in range(B)])
    rewards = torch.randn(B, R) * (torch.rand(B, R) > 0.8)
    mask = (torch.rand(B, R) > 0.2).float()
    want, _ = ref.compute_rloo_outcome_advantage(rewards.clone(), mask, index)
    from verl_amd import _lib as L

    got = K.outcome_advantage(rewards.to(DEV), mask.to(DEV), index, 1e-6, L.VA_ADV_RLOO)
    _close(got, want, atol=1e-5, rtol=1e-5, what="rloo")


@pytest.mark.parametrize("R", [1, 17, 64, 65, 256, 513, 1024, 1025, 3000, 20000])
@pytest.mark.parametrize("gamma,lam", [(1.0, 1.0), (0.99, 0.95)])
def test_gae_matches_oracle(K, R, gamma, lam):
    torch.manual_seed(R)
    B = 33
    rewards = torch.randn(B, R) * (torch.rand(B, R) > 0.9)
    values = torch.randn(B, R)
    lens = torch.randint(1, R + 1, (B,))
    mask = (torch.arange(R)[None, :] < lens[:, None]).to(torch.int64)
    if R > 2:
        mask[1] = (torch.rand(R) > 0.5).long()  # multi-turn style holes
        mask[1, 0] = 1
    want_adv, want_ret = ref.compute_gae_advantage_return(rewards.double(), values.double(), mask.double(), gamma, lam)
    adv, ret = K.gae_advantage_return(rewards.to(DEV), values.to(DEV), mask.to(DEV), gamma, lam)
    # error budget vs the float64 twin: the recurrence is reassociated into a chunked scan
    tol = 1e-4 * max(1.0, float(np.sqrt(R) / 8))
    _close(ret, want_ret, atol=tol, rtol=1e-4, what="gae returns")
    _close(adv, want_adv, atol=tol, rtol=1e-4, what="gae advantages")


@pytest.mark.parametrize("B,R", [(7, 1), (33, 65), (512, 1024), (9, 1000)])
def test_gae_register_and_lds_kernels_agree(K, B, R):
    """The register-chunk and LDS-staged scans use the same chunking and op order: returns are
    bitwise equal; whitened advantages differ at most by the fp64 partials' summation order."""
    from verl_amd import _lib as L

    torch.manual_seed(B + R)
    rewards = (torch.randn(B, R) * (torch.rand(B, R) > 0.9)).to(DEV)
    values = torch.randn(B, R).to(DEV)
    lens = torch.randint(1, R + 1, (B,))
    mask = (torch.arange(R)[None, :] < lens[:, None]).to(torch.int64).to(DEV)
    outs = []
    try:
        for variant in (1, 2):
            L.call("va_set_tuning", L.VA_TUNE_GAE_VARIANT, variant)
            outs.append(K.gae_advantage_return(rewards, values, mask, 0.99, 0.95))
    finally:
        L.call("va_set_tuning", L.VA_TUNE_GAE_VARIANT, 0)
    assert torch.equal(outs[0][1], outs[1][1])
    _close(outs[0][0], outs[1][0].cpu(), atol=1e-6, rtol=1e-6, what="gae adv reg vs lds")


def test_gae_multi_turn_property(K):
    """tests/trainer/ppo/test_core_algos_on_cpu.py:134-188: advantages and masked returns do not
    depend on values at mask == 0 positions (bit-identical)."""
    import random

    random.seed(0)
    gamma, lam = random.uniform(0, 1), random.uniform(0, 1)
    rewards = torch.tensor([[0.0, 0.0, 0.1, 0.1, 0.1, 0.0, 0.0, 0.1, 1.0, 0.0, 0.0]])
    v1 = torch.tensor([[random.uniform(-100, 100), random.random(), 4.0, 5.0, 6.0, random.uniform(-100, 0),
                        random.random(), 7.0, 9.0, 0.0, 0.0]])
    v2 = torch.tensor([[random.random(), random.uniform(-100, 100), 4.0, 5.0, 6.0, random.random(),
                        random.uniform(0, 100), 7.0, 9.0, 0.0, 0.0]])
    mask = torch.tensor([[0, 0, 1, 1, 1, 0, 0, 1, 1, 0, 0]], dtype=torch.float)
    a1, r1 = K.gae_advantage_return(rewards.to(DEV), v1.to(DEV), mask.to(DEV), gamma, lam)
    a2, r2 = K.gae_advantage_return(rewards.to(DEV), v2.to(DEV), mask.to(DEV), gamma, lam)
    m = mask.to(DEV)
    assert torch.equal(a1, a2)
    assert torch.equal(r1 * m, r2 * m)
    want_a, _ = ref.compute_gae_advantage_return(rewards, v1, mask, gamma, lam)
    _close(a1, want_a, atol=1e-5, what="multi-turn adv")


def test_gae_mask_errors(K):
    r = torch.zeros(2, 5, device=DEV)
    with pytest.raises(ValueError, match="At least one element"):
        K.gae_advantage_return(r, r, torch.zeros(2, 5, device=DEV), 1.0, 1.0)
    m = torch.zeros(2, 5, device=DEV)
    m[0, 0] = 1
    with pytest.raises(ValueError, match="sum of the mask is one"):
        K.gae_advantage_return(r, r, m, 1.0, 1.0)


def test_whiten_matches_oracle(K):
    torch.manual_seed(1)
    x = torch.randn(50, 123) * 3 + 1
    mask = (torch.rand(50, 123) > 0.4).float()
    stats, merged = K.whiten_stats(x.to(DEV), mask.to(DEV))
    got = K.whiten_apply(x.to(DEV), mask.to(DEV), stats)
    _close(got, ref.masked_whiten(x.double(), mask.double()), atol=1e-5, what="whiten")


def test_apply_kl_penalty(K):
    torch.manual_seed(6)
    B, R = 16, 90
    scores = torch.zeros(B, R)
    scores[:, -1] = torch.rand(B)
    old = -torch.rand(B, R)
    refl = old + torch.randn(B, R) * 0.1
    mask = (torch.rand(B, R) > 0.3).long()
    want_r, want_kl = ref.apply_kl_penalty(scores, old, refl, mask, beta=0.05, kl_type="low_var_kl")
    got_r, row_kl = K.apply_kl_penalty(scores.to(DEV), old.to(DEV), refl.to(DEV), mask.to(DEV), 0.05, "low_var_kl")
    _close(got_r, want_r, atol=1e-6, what="kl rewards")
    assert abs(row_kl.mean().item() - want_kl) < 1e-6


@pytest.mark.parametrize("B,R", [(8192, 1024), (5, 1000), (3, 2048), (6, 260)])
def test_gae_quad_kernel_vs_float64_twin(K, B, R):
    """The quad-streaming scan (default where R % 4 == 0, R <= 2048) against the fp64 oracle at
    16x the headline batch and at ragged shapes (R not a multiple of 256, partial workgroups)."""
    g = torch.Generator().manual_seed(B * 7 + R)
    rewards = torch.randn(B, R, generator=g) * (torch.rand(B, R, generator=g) > 0.9)
    values = torch.randn(B, R, generator=g)
    lens = torch.randint(1, R + 1, (B,), generator=g)
    mask = (torch.arange(R)[None, :] < lens[:, None]).to(torch.int64)
    mask[0] = (torch.rand(R, generator=g) > 0.5).long()  # multi-turn holes
    want_adv, want_ret = ref.compute_gae_advantage_return(rewards.double(), values.double(), mask.double(), 0.99, 0.95)
    adv, ret = K.gae_advantage_return(rewards.to(DEV), values.to(DEV), mask.to(DEV), 0.99, 0.95)
    tol = 1e-4 * max(1.0, float(np.sqrt(R) / 8))
    _close(ret, want_ret, atol=tol, rtol=1e-4, what="gae quad returns")
    _close(adv, want_adv, atol=tol, rtol=1e-4, what="gae quad advantages")


def test_gae_quad_kernel_multi_turn_property(K):
    """The multi-turn property (values at mask == 0 do not matter, bitwise) on the quad kernel."""
    g = torch.Generator().manual_seed(3)
    B, R = 16, 1024
    rewards = torch.randn(B, R, generator=g) * (torch.rand(B, R, generator=g) > 0.9)
    mask = (torch.rand(B, R, generator=g) > 0.4).float()
    v1 = torch.randn(B, R, generator=g)
    v2 = torch.where(mask > 0, v1, torch.randn(B, R, generator=g) * 100)
    a1, r1 = K.gae_advantage_return(rewards.to(DEV), v1.to(DEV), mask.to(DEV), 0.97, 0.9)
    a2, r2 = K.gae_advantage_return(rewards.to(DEV), v2.to(DEV), mask.to(DEV), 0.97, 0.9)
    m = mask.to(DEV)
    assert torch.equal(a1, a2)
    assert torch.equal(r1 * m, r2 * m)


@pytest.mark.parametrize("with_entropy", [True, False])
@pytest.mark.parametrize("R", [1024, 1000, 2048, 260, 17])
@pytest.mark.parametrize("mode", ["vanilla", "gpg", "clip_cov", "kl_cov"])
def test_policy_loss_streaming_forward_matches_workgroup_kernel(K, R, mode, with_entropy):
    """VA_TUNE_LOSS_VEC: the wave-per-row streaming forward (default where it applies) and the
    workgroup-per-row forward give the same 8 slots (fp64 row sums in another order) and bitwise
    the same gradients (the backward reads only counts from the partials). Covers the four
    instances of the streaming kernel's compile-time optional inputs (entropy rows x selection)."""
    from verl_amd import _lib as L

    g = torch.Generator().manual_seed(R)
    B = 37
    old = (-torch.rand(B, R, generator=g) * 3).to(DEV)
    lp = (old.cpu() + 0.3 * torch.randn(B, R, generator=g)).to(DEV)
    adv = torch.randn(B, R, generator=g).to(DEV)
    ref_ = (old.cpu() + 0.1 * torch.randn(B, R, generator=g)).to(DEV)
    ent = torch.rand(B, R, generator=g).to(DEV)
    lens = torch.randint(1, R + 1, (B,), generator=g)
    mask = (torch.arange(R)[None, :] < lens[:, None]).long().to(DEV)
    sel = (torch.rand(B, R, generator=g) < 0.05).to(DEV) if mode in ("clip_cov", "kl_cov") else None
    outs = []
    try:
        for v in (1, 0):
            L.call("va_set_tuning", L.VA_TUNE_LOSS_VEC, v)
            x = lp.clone().requires_grad_(True)
            e = ent.clone().requires_grad_(True) if with_entropy else None
            out = K.fused_policy_loss(old, x, adv, mask, 0.2, 0.28, 3.0, "token-mean", ref_log_prob=ref_,
                                      kl_loss_type="low_var_kl", entropy=e, loss_mode=mode, selection=sel,
                                      mode_coef=0.1)
            (out[0] + 0.01 * out[4] - 0.001 * out[5]).backward()
            outs.append((out.detach().cpu(), x.grad.cpu(), e.grad.cpu() if with_entropy else None))
    finally:
        L.call("va_set_tuning", L.VA_TUNE_LOSS_VEC, 1)
    _close(outs[0][0], outs[1][0], atol=1e-6, rtol=1e-6, what="loss slots vec vs wg")
    assert torch.equal(outs[0][1], outs[1][1])
    if with_entropy:
        assert torch.equal(outs[0][2], outs[1][2])
    else:
        assert outs[0][0][5].item() == 0.0  # the entropy slot of a loss without entropy rows


@pytest.mark.parametrize("B", [1500, 4500, 9001])
@pytest.mark.parametrize("agg", ["token-mean", "seq-mean-token-sum", "seq-mean-token-mean", "seq-mean-token-sum-norm"])
def test_policy_loss_multi_row_workgroups_match_workgroup_kernel(K, B, agg):
    """Large batches: the streaming forward's 4-row workgroups (ragged last workgroup) fold each
    row's per-row aggregate into one vector per workgroup for the finalize (up to 2,251 vectors,
    several load rounds of the 1,024-thread finalize); every loss slot equals the
    workgroup-per-row kernel's up to fp64 summation order, for every aggregation mode."""
    from verl_amd import _lib as L

    R = 512
    g = torch.Generator(device=DEV).manual_seed(B)
    old = -torch.rand(B, R, device=DEV, generator=g) * 3
    lp = old + 0.3 * torch.randn(B, R, device=DEV, generator=g)
    adv = torch.randn(B, R, device=DEV, generator=g)
    ref_ = old + 0.1 * torch.randn(B, R, device=DEV, generator=g)
    ent = torch.rand(B, R, device=DEV, generator=g)
    lens = torch.randint(1, R + 1, (B,), device=DEV, generator=g)  # seq-mean-token-mean: 0/0 rows are NaN
    mask = (torch.arange(R, device=DEV)[None, :] < lens[:, None]).to(torch.bool)
    outs = []
    try:
        for vec in (0, 1):
            L.call("va_set_tuning", L.VA_TUNE_LOSS_VEC, vec)
            out = K.fused_policy_loss(old, lp, adv, mask, 0.2, 0.28, 3.0, agg, ref_log_prob=ref_,
                                      kl_loss_type="low_var_kl", entropy=ent)
            outs.append(out.detach().cpu())
    finally:
        L.call("va_set_tuning", L.VA_TUNE_LOSS_VEC, 1)
    for o in outs[1:]:
        _close(o, outs[0], atol=1e-6, rtol=1e-6, what=f"loss slots multi-row vs wg ({agg}, B={B})")
