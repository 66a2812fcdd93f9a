"""va_transpose_16 (model_ops.hip) and the transposed-weight input gradient (kernels.input_grad):
the transpose is bit-exact against torch's copy for partial tiles, row-strided input, the
lm_head's 151,936 x 896 weight and both 16-bit types; the TN input gradient equals the plain
product to bf16 rounding (same fp32 accumulation, another kernel order), and the lm_head / linear
autograd through kernels.linear matches nn.Linear's."""

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("R,C", [(8, 8), (64, 64), (136, 200), (896, 9728), (4864, 896), (151936, 896)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_transpose16_bit_exact(R, C, dtype):
    from verl_amd import kernels as K

    x = torch.randn(R, C, device=DEV).to(dtype)
    out = K.transpose16(x)
    assert out.shape == (C, R) and out.is_contiguous()
    assert torch.equal(out, x.t().contiguous())


def test_transpose16_row_strided_input():
    from verl_amd import kernels as K

    base = torch.randn(200, 264, device=DEV).to(torch.bfloat16)
    x = base[:, 8:208]  # ld 264, 16-byte aligned start
    assert x.stride(0) == 264 and x.data_ptr() % 16 == 0
    assert torch.equal(K.transpose16(x), x.t().contiguous())


def test_input_grad_tn_matches_plain_product():
    from verl_amd import kernels as K

    g = torch.Generator(device=DEV).manual_seed(3)
    for n_out, n_in in [(9728, 896), (896, 4864), (1152, 896)]:
        w = (torch.randn(n_out, n_in, device=DEV, generator=g) * 0.02).to(torch.bfloat16)
        dy = torch.randn(4096, n_out, device=DEV, generator=g).to(torch.bfloat16)
        ref = dy.float() @ w.float()
        got = K.input_grad(dy, w).float()
        # fp32 accumulation in both layouts; the output is rounded to bf16 once (2^-8 relative)
        tol = 2.0 ** -7 * ref.abs().max().item()
        assert (got - ref).abs().max().item() <= tol
        assert (got - (dy @ w).float()).abs().max().item() <= tol


def test_linear_autograd_matches_nn_linear():
    from verl_amd import kernels as K

    torch.manual_seed(0)
    head = torch.nn.Linear(896, 4096, bias=False, device=DEV, dtype=torch.bfloat16)
    x = torch.randn(2048, 896, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    g = torch.randn(2048, 4096, device=DEV, dtype=torch.bfloat16)
    y_ref = head(x)
    y_ref.backward(g)
    dx_ref, dw_ref = x.grad.clone(), head.weight.grad.clone()
    x.grad, head.weight.grad = None, None
    y = K.linear(x, head.weight)
    assert torch.equal(y, y_ref)  # the same forward GEMM
    y.backward(g)
    scale_x, scale_w = dx_ref.float().abs().max().item(), dw_ref.float().abs().max().item()
    assert (x.grad.float() - dx_ref.float()).abs().max().item() <= 2.0 ** -7 * scale_x
    assert (head.weight.grad.float() - dw_ref.float()).abs().max().item() <= 2.0 ** -7 * scale_w


def test_weight_grad_swapped_order_for_vocab_sized_outputs():
    """n_out >= WGRAD_SWAP_MIN_OUT (the lm_head): dW = (X^T dY)^T through va_transpose_16."""
    from verl_amd import kernels as K

    g = torch.Generator(device=DEV).manual_seed(5)
    n_out = K.WGRAD_SWAP_MIN_OUT + 64
    dy = torch.randn(3000, n_out, device=DEV, generator=g).to(torch.bfloat16)
    x = torch.randn(3000, 136, device=DEV, generator=g).to(torch.bfloat16)
    got = K.weight_grad(dy, x)
    assert got.shape == (n_out, 136) and got.is_contiguous()
    ref = dy.float().t() @ x.float()
    assert (got.float() - ref).abs().max().item() <= 2.0 ** -7 * ref.abs().max().item()
    assert (got.float() - (dy.t() @ x).float()).abs().max().item() <= 2.0 ** -7 * ref.abs().max().item()
