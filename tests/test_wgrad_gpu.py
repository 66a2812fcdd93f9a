"""gfx950 weight-gradient kernel (wgrad.hip) against an fp32 torch reference of dW = dY^T X."""

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("T,M,N,splits", [(64, 128, 128, 1), (1000, 256, 384, 1), (4097, 1152, 896, 4),
                                          (3000, 896, 4864, 3), (777, 9728, 896, 2), (130, 128, 256, 8)])
def test_wgrad_matches_fp32_reference(T, M, N, splits):
    from verl_amd import kernels as K

    torch.manual_seed(T + M)
    dy = torch.randn(T, M, device=DEV).to(torch.bfloat16)
    x = torch.randn(T, N, device=DEV).to(torch.bfloat16)
    got = K.wgrad_gemm(dy, x, splits)
    want = dy.float().t() @ x.float()
    err = (got.float() - want).abs()
    tol = 2 ** -7 * want.abs() + 1e-2 * (T ** 0.5)
    assert torch.all(err <= tol), f"max err {err.max().item():.3e}"


def test_wgrad_strided_rows_and_split_equivalence():
    """Row strides (views of merged buffers) and any split count give the fp32 sum rounded once:
    splits differ only in fp32 summation order."""
    from verl_amd import kernels as K

    torch.manual_seed(3)
    big = torch.randn(2048, 1152 + 128, device=DEV).to(torch.bfloat16)
    dy = big[:, :1152]
    x = torch.randn(2048, 896, device=DEV).to(torch.bfloat16)
    a = K.wgrad_gemm(dy, x, 1).float()
    b = K.wgrad_gemm(dy, x, 4).float()
    want = dy.float().t() @ x.float()
    assert torch.all((a - want).abs() <= 2 ** -7 * want.abs() + 1e-2)
    assert (a - b).abs().max().item() <= 2 ** -7 * want.abs().max().item()
