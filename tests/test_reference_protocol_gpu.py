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
This pins the log-prob / entropy restatement to torch itself, independently of the oracle.
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
