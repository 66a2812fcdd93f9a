"""The fused backward's dlogits kernel (va_linear_logprob_bwd, linear_logprob.hip) at kernel level: bitwise
against the unfused composition on exact-arithmetic logits, and per vocabulary range against the
whole-vocabulary launch. One backward kernel: unlike test_linear_logprob_gpu.py these do not run per
forward tile setting."""

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _exact_inputs(N, H, V, seed):
    g = torch.Generator().manual_seed(seed)
    h = (torch.randint(-4, 5, (N, H), generator=g).float() / 8).to(torch.bfloat16)
    w = (torch.randint(-4, 5, (V, H), generator=g).float() / 16).to(torch.bfloat16)
    return h, w


@pytest.mark.parametrize("N,H,V", [(300, 64, 1000), (256, 896, 151936), (77, 128, 36), (1, 64, 132)])
@pytest.mark.parametrize("T", [1.0, 0.7])
@pytest.mark.parametrize("ent_grad", [False, True])
def test_fused_backward_dlogits_bitwise_on_exact_logits(N, H, V, T, ent_grad):
    """the fused backward recomputes the logits inside its MFMA tiles and forms
    dlogits in registers. On exact-arithmetic data (every GEMM order gives the same logits) its bf16
    dlogits equal bitwise those of the unfused composition — bf16 logits in HBM, then the streaming
    va_logprob_entropy_bwd — given the same (lse, entropy) and upstream gradients, including
    ignore_index / out-of-range labels, rows past a 256-row block and vocab tails."""
    from verl_amd import kernels as K

    h, w = _exact_inputs(N, H, V, seed=N * 3 + V)
    g = torch.Generator().manual_seed(N + H)
    labels = torch.randint(0, V, (N,), generator=g)
    if N > 2:
        labels[0], labels[1] = -100, V + 3
    labels[-1] = V - 1
    logits = (h.float() @ w.float().t()).to(torch.bfloat16).to(DEV)  # exact fp32 sums, one rounding
    h, w, labels = h.to(DEV), w.to(DEV), labels.to(DEV)
    _, ent, lse = torch.ops.verl_amd.logprob_entropy_fwd(logits, labels, T, 0)
    g1 = torch.randn(N, generator=g).to(DEV)
    g2 = torch.randn(N, generator=g).to(DEV) if ent_grad else None
    want = torch.ops.verl_amd.logprob_entropy_bwd(g1, g2, logits, labels, lse, ent, T)
    got = torch.full((N, V + 4), 7.0, dtype=torch.bfloat16, device=DEV)[:, :V]  # row stride > V
    K._linear_logprob_bwd_raw(h, w, labels, lse, ent, g1, g2, T, False, got)
    assert torch.equal(torch.isnan(got), torch.isnan(want))
    assert torch.equal(torch.nan_to_num(got), torch.nan_to_num(want)), (got.float() - want.float()).abs().max()


@pytest.mark.parametrize("N,H,V,bounds", [
    (300, 64, 1000, [0, 300, 604, 1000]),       # ranges not multiples of the 256-wide tile
    (256, 896, 151936, list(range(0, 151936, 9504)) + [151936]),  # the reference's vocab_per_split
    (77, 128, 38, [0, 4, 36, 38]),              # V % 4 != 0: every range but the last is a multiple of 4
])
@pytest.mark.parametrize("T", [1.0, 0.7])
def test_vocab_range_dlogits_equal_the_whole_vocab_launch(N, H, V, bounds, T):
    """ABI 6: va_linear_logprob_bwd over vocab ranges [v0, v1) writes exactly the columns v0..v1 of
    the whole-vocabulary launch, bitwise: the labels (ignore_index, out of range, in every range)
    and the g_logp term of the softmax gradient count against the whole vocabulary. Where V % 4 != 0
    the whole launch is not allowed, so the last 2 columns are compared with the unfused
    composition."""
    from verl_amd import kernels as K

    h, w = _exact_inputs(N, H, V, seed=N + 2 * V)
    g = torch.Generator().manual_seed(V)
    labels = torch.randint(0, V, (N,), generator=g)
    labels[0], labels[1], labels[2] = -100, V + 3, V - 1
    logits = (h.float() @ w.float().t()).to(torch.bfloat16).to(DEV)
    h, w, labels = h.to(DEV), w.to(DEV), labels.to(DEV)
    _, ent, lse = torch.ops.verl_amd.logprob_entropy_fwd(logits, labels, T, 0)
    g1, g2 = torch.randn(N, generator=g).to(DEV), torch.randn(N, generator=g).to(DEV)
    want = torch.ops.verl_amd.logprob_entropy_bwd(g1, g2, logits, labels, lse, ent, T)
    if V % 4 == 0:
        whole = torch.empty(N, V, dtype=torch.bfloat16, device=DEV)
        K._linear_logprob_bwd_raw(h, w, labels, lse, ent, g1, g2, T, False, whole)
        assert torch.equal(torch.nan_to_num(whole), torch.nan_to_num(want))
    for v0, v1 in zip(bounds[:-1], bounds[1:]):
        if (v1 - v0) % 4:
            continue
        part = torch.full((N, v1 - v0 + 8), 7.0, dtype=torch.bfloat16, device=DEV)[:, : v1 - v0]
        K._linear_logprob_bwd_raw(h, w, labels, lse, ent, g1, g2, T, False, part, v0, v1)
        assert torch.equal(torch.nan_to_num(part), torch.nan_to_num(want[:, v0:v1])), (v0, v1)


@pytest.mark.parametrize("defer", [0, 2])
@pytest.mark.parametrize("N,H,V,ldd", [(300, 896, 151936, 151936), (77, 128, 1000, 1008), (513, 64, 2048, 2052)])
def test_dlogits_epilogue_placement_bitwise(defer, N, H, V, ldd):
    """VA_TUNE_T256_DEFER bit 2: the dlogits tile epilogue before or after the step's operand wait
    (16-byte rows through the scratch, and 8-byte stores when ldd % 8 != 0) writes the unfused
    composition's dlogits bit for bit on exact data."""
    from verl_amd import _lib as L
    from verl_amd import kernels as K

    h, w = _exact_inputs(N, H, V, seed=N + V + ldd)
    g = torch.Generator().manual_seed(N)
    labels = torch.randint(0, V, (N,), generator=g)
    labels[0] = -100
    logits = (h.float() @ w.float().t()).to(torch.bfloat16).to(DEV)
    h, w, labels = h.to(DEV), w.to(DEV), labels.to(DEV)
    _, ent, lse = torch.ops.verl_amd.logprob_entropy_fwd(logits, labels, 1.0, 0)
    g1, g2 = torch.randn(N, generator=g).to(DEV), torch.randn(N, generator=g).to(DEV)
    want = torch.ops.verl_amd.logprob_entropy_bwd(g1, g2, logits, labels, lse, ent, 1.0)
    got = torch.full((N, ldd), 7.0, dtype=torch.bfloat16, device=DEV)
    try:
        L.call("va_set_tuning", L.VA_TUNE_T256_DEFER, defer)
        K._linear_logprob_bwd_raw(h, w, labels, lse, ent, g1, g2, 1.0, False, got[:, :V])
    finally:
        L.call("va_set_tuning", L.VA_TUNE_T256_DEFER, 1)
    assert torch.equal(torch.nan_to_num(got[:, :V]), torch.nan_to_num(want))
    assert (got[:, V:].float() == 7.0).all()


def test_epilogue_placement_key_range():
    from verl_amd import _lib as L

    with pytest.raises(RuntimeError, match="VA_TUNE_T256_DEFER"):
        L.call("va_set_tuning", L.VA_TUNE_T256_DEFER, 8)
