"""The reference's own log-prob / entropy test protocol, run against this build's kernels.

Reference: tests/utils/test_linear_cross_entropy.py (GPU-only there). Same three shapes
(:115-130: 1937 x 3584 x 152064, 2169 x 896 x 151936 — Qwen2.5-0.5B's lm_head — and
1530 x 2048 x 32256), same inputs (:145-161: bf16 hidden / weight ~ U(-0.5, 0.5), labels
U[0, V), temperature 1.5, g_entropy ~ U(-0.5, 0.5), g_logprobs ~ U(-1, 1)), same independent
reference (:47-59 `run_torch_entropy`: fp32 logits, -F.cross_entropy, logsumexp - sum(softmax * x)),
and the reference's own tolerances:
  * the unfused path (fp32 logits -> logprobs_from_logits / entropy_from_logits, the product's
    streaming kernel): 1e-4 / 1e-4 forward (:210-211), 1e-2 / 1e-4 gradients (:258-259);
  * the fused lm_head kernel (no logits in HBM) in its fp32-logits mode — the reference's fused
    kernel keeps the logits fp32; the default mode rounds them to bf16 like the unfused autocast
    path — 1e-3 / 2e-4 log-probs, 5e-3 / 5e-4 entropy (:217-218), 2e-2 / 4e-2 gradients (:267-268).
This pins the log-prob / entropy restatement to torch itself, independently of the oracle; the
fused kernel's default (bf16-logits) mode is pinned to an fp32 torch reference with the same two
bf16 roundings (test_fused_lm_head_default_mode_against_torch).
"""

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
TEMPERATURE = 1.5
CASES = [(1937, 3584, 152064), (2169, 896, 151936), (1530, 2048, 32256)]


def _inputs(N, H, V, seed):
    torch.manual_seed(seed)
    hidden = torch.empty(N, H, dtype=torch.bfloat16, device=DEV).uniform_(-0.5, 0.5).requires_grad_(True)
    weight = torch.empty(V, H, dtype=torch.bfloat16, device=DEV).uniform_(-0.5, 0.5).requires_grad_(True)
    labels = torch.randint(0, V, (N,), device=DEV)
    g_ent = torch.empty(N, dtype=torch.bfloat16, device=DEV).uniform_(-0.5, 0.5)
    g_lp = torch.empty(N, dtype=torch.bfloat16, device=DEV).uniform_(-1, 1)
    return hidden, weight, labels, g_ent, g_lp


def _torch_reference(hidden, weight, labels, T):
    logits = hidden.float() @ weight.float().t()
    logits = logits / T
    pd = torch.softmax(logits, dim=-1)
    entropy = torch.logsumexp(logits, dim=-1) - (pd * logits).sum(-1)
    logprobs = -torch.nn.functional.cross_entropy(logits, labels, reduction="none")
    return logprobs, entropy


def _grads(outs, leaves, g_ent, g_lp):
    lp, ent = outs
    return torch.autograd.grad((ent, lp), leaves, (g_ent.to(ent.dtype), g_lp.to(lp.dtype)))


@pytest.mark.parametrize("N,H,V", CASES)
def test_streaming_logprob_kernel_reference_protocol(N, H, V):
    from verl_amd import kernels as K

    hidden, weight, labels, g_ent, g_lp = _inputs(N, H, V, seed=N)
    want = _torch_reference(hidden, weight, labels, TEMPERATURE)
    logits = hidden.float() @ weight.float().t()
    got = K.logprob_entropy(logits, labels, temperature=TEMPERATURE)
    torch.testing.assert_close(got[0], want[0], atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(got[1], want[1], atol=1e-4, rtol=1e-4)
    dh_w, dw_w = _grads(want, (hidden, weight), g_ent, g_lp)
    dh_g, dw_g = _grads(got, (hidden, weight), g_ent, g_lp)
    torch.testing.assert_close(dh_g, dh_w, atol=1e-2, rtol=1e-4)
    torch.testing.assert_close(dw_g, dw_w, atol=1e-2, rtol=1e-4)


@pytest.mark.parametrize("tile", [256, 128])
@pytest.mark.parametrize("N,H,V", CASES)
def test_fused_lm_head_kernel_reference_protocol(N, H, V, tile):
    from verl_amd import _lib as L
    from verl_amd import kernels as K

    L.call("va_set_tuning", L.VA_TUNE_LINEAR_LOGPROB_TILE, tile)
    try:
        _fused_case(K, N, H, V)
    finally:
        L.call("va_set_tuning", L.VA_TUNE_LINEAR_LOGPROB_TILE, 256)


def _fused_case(K, N, H, V):
    hidden, weight, labels, g_ent, g_lp = _inputs(N, H, V, seed=N + 1)
    want = _torch_reference(hidden, weight, labels, TEMPERATURE)
    got = K.linear_logprob_entropy(hidden, weight, labels, TEMPERATURE, fp32_logits=True)
    torch.testing.assert_close(got[0], want[0], atol=1e-3, rtol=2e-4)
    torch.testing.assert_close(got[1], want[1], atol=5e-3, rtol=5e-4)
    dh_w, dw_w = _grads(want, (hidden, weight), g_ent, g_lp)
    dh_g, dw_g = _grads(got, (hidden, weight), g_ent, g_lp)
    torch.testing.assert_close(dh_g, dh_w, atol=2e-2, rtol=4e-2)
    torch.testing.assert_close(dw_g, dw_w, atol=2e-2, rtol=4e-2)


def _st_round(x):
    """bf16 rounding with an identity gradient: the autocast path's bf16 logits and div_(T)
    (dp_actor.py:182) as torch autograd sees them (the rounding is not differentiated)."""
    return x + (x.to(torch.bfloat16).float() - x).detach()


@pytest.mark.parametrize("N,H,V", [(2169, 896, 151936)])
def test_fused_lm_head_default_mode_against_torch(N, H, V):
    """The fused lm_head kernel in its DEFAULT mode (logits rounded to bf16, then bf16(x / T), as
    the unfused autocast path holds them) pinned to torch itself: an fp32 reference with the same
    two roundings (straight-through in the backward), on the reference protocol's inputs. What
    remains is the accumulation order of the fp32 dot products before rounding (MFMA tiles vs
    torch's GEMM), which can move a logit by one bf16 unit: bounds of one unit at |x| < 8 (2^-5)
    for a row's log-prob, 1e-3 on entropy, and 1e-2 relative L2 on both gradients (dlogits are
    bf16 for the lm_head GEMMs, as under autocast)."""
    from verl_amd import kernels as K

    hidden, weight, labels, g_ent, g_lp = _inputs(N, H, V, seed=N + 7)
    h32 = hidden.detach().float().requires_grad_(True)
    w32 = weight.detach().float().requires_grad_(True)
    x = _st_round(_st_round(h32 @ w32.t()) / TEMPERATURE)
    want = (torch.log_softmax(x, dim=-1).gather(-1, labels[:, None])[:, 0],
            torch.logsumexp(x, dim=-1) - (torch.softmax(x, dim=-1) * x).sum(-1))
    got = K.linear_logprob_entropy(hidden, weight, labels, TEMPERATURE)
    dlp = (got[0] - want[0]).abs()
    assert dlp.max().item() <= 2 ** -5 and dlp.mean().item() < 1e-4, (dlp.max().item(), dlp.mean().item())
    assert (got[1] - want[1]).abs().max().item() < 1e-3
    dh_w, dw_w = torch.autograd.grad((want[1], want[0]), (h32, w32), (g_ent.float(), g_lp.float()))
    dh_g, dw_g = _grads(got, (hidden, weight), g_ent, g_lp)
    for g, w, what in ((dh_g, dh_w, "d_hidden"), (dw_g, dw_w, "d_weight")):
        err = ((g.float() - w).norm() / w.norm()).item()
        assert err < 1e-2, f"{what}: relative L2 error {err:.3e}"
