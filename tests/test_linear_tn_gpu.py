"""va_linear_tn (csrc/gemm_tn.hip): y = bf16(x w^T + b), the backbone projections' F.linear (torch's
nn.Linear in the reference, dp_actor.py:331-333 / :465-470). On exact-arithmetic operands (small
integers: every fp32 partial sum exact, whatever the order) bitwise equal to F.linear (hipBLASLt); on
random operands within the fp32-accumulation tolerance of an fp32 product; tails (rows past a 256-token
block), strided operands, every tile width, explicit tiles-per-workgroup and the argument checks."""

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _run(x, w, b=None, tile=0, per=0, ldy=None):
    from verl_amd import _lib as L
    from verl_amd import kernels as K

    M, Kd = x.shape
    N = w.shape[0]
    ldy = ldy or N
    buf = torch.full((M, ldy), float("nan"), dtype=torch.bfloat16, device=DEV)
    L.call("va_linear_tn", K._p(x), x.stride(0), K._p(w), w.stride(0), K._p(b) if b is not None else None, L.VA_BF16,
           M, N, Kd, tile, per, K._p(buf), ldy, K._stream(x))
    return buf[:, :N], buf


def _ints(shape, lo, hi, gen, scale=1.0):
    return (torch.randint(lo, hi + 1, shape, device=DEV, generator=gen).float() * scale).to(torch.bfloat16)


@pytest.mark.parametrize("M,N,K,tile,bias", [
    (512, 896, 896, 0, False), (300, 896, 1152, 0, False), (1, 896, 896, 0, False), (777, 1152, 896, 0, True),
    (256, 1152, 896, 192, True), (513, 768, 256, 256, False), (1024, 896, 4864, 224, False), (96, 576, 128, 288, False),
    (2048, 1152, 640, 288, True)])
def test_exact_operands_bitwise_equal_to_f_linear(M, N, K, tile, bias):
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    x = _ints((M, K), -3, 3, g)
    w = _ints((N, K), -3, 3, g, 0.25)
    b = _ints((N,), -20, 20, g, 0.5) if bias else None
    y, _ = _run(x, w, b, tile=tile)
    ref = torch.nn.functional.linear(x, w, b)
    assert torch.equal(y, ref)


@pytest.mark.parametrize("mode", [2, 1])
@pytest.mark.parametrize("M,N,K,bias", [(257, 896, 128, True), (1000, 1152, 1152, True), (3000, 896, 4864, False),
                                         (2560, 896, 896, False), (600, 896, 192, False), (513, 1152, 256, True)])
def test_forms_bitwise_equal_on_exact_data(mode, M, N, K, bias):
    """The ping-pong form (K >= 192: its rings run on across tiles) and the two-buffer form, per tile
    boundary / row tail / per-workgroup tile count."""
    from verl_amd import _lib as L

    g = torch.Generator(device=DEV).manual_seed(M * 7 + K)
    x = _ints((M, K), -3, 3, g)
    w = _ints((N, K), -3, 3, g, 0.25)
    b = _ints((N,), -20, 20, g, 0.5) if bias else None
    ref = torch.nn.functional.linear(x, w, b)
    try:
        L.call("va_set_tuning", L.VA_TUNE_LINEAR_TN, mode)
        for per in (0, 1, 2, 5):
            y, _ = _run(x, w, b, per=per)
            assert torch.equal(y, ref), per
    finally:
        L.call("va_set_tuning", L.VA_TUNE_LINEAR_TN, 2)


@pytest.mark.parametrize("M,N,K,bias", [(4096, 896, 896, False), (3000, 1152, 896, True), (2048, 896, 9728, False)])
def test_random_operands_within_fp32_accumulation_tolerance(M, N, K, bias):
    g = torch.Generator(device=DEV).manual_seed(7)
    x = torch.randn(M, K, device=DEV, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV, generator=g) * 0.03).to(torch.bfloat16)
    b = (torch.randn(N, device=DEV, generator=g) * 0.1).to(torch.bfloat16) if bias else None
    y, _ = _run(x, w, b)
    ref = torch.nn.functional.linear(x.float(), w.float(), b.float() if b is not None else None)
    # the one bf16 rounding (2^-9 relative) plus the fp32 summation-order difference
    err = (y.float() - ref).abs()
    assert (err <= ref.abs() * 2.0 ** -8 + 1e-3).all(), err.max().item()
    blas = torch.nn.functional.linear(x, w, b)
    assert (y.float() - blas.float()).norm() / blas.float().norm() < 2e-3


def test_strided_operands_tiles_per_workgroup_and_row_stride():
    g = torch.Generator(device=DEV).manual_seed(3)
    xs = _ints((700, 1024), -3, 3, g)[:, 64:960]  # ldx 1024, K 896
    ws = _ints((896, 1152), -3, 3, g, 0.5)[:, :896]  # ldw 1152
    ref = torch.nn.functional.linear(xs, ws)
    from verl_amd import _lib as L

    try:
        for order in (2, 1, 0):  # VA_TUNE_LINEAR_TN: the ping-pong form, the two-buffer form's two tile orders
            L.call("va_set_tuning", L.VA_TUNE_LINEAR_TN, order)
            for per in (0, 1, 3, 7, 100):
                y, buf = _run(xs, ws, per=per, ldy=904)
                assert torch.equal(y, ref), (order, per)
                assert torch.isnan(buf[:, 896:].float()).all()  # nothing written past N
    finally:
        L.call("va_set_tuning", L.VA_TUNE_LINEAR_TN, 2)


def test_bench_shape_o_projection_bitwise_on_exact_data():
    """The bench's packed update pass (151,552 tokens) on the o projection: 592 token blocks x 4 tiles over
    the persistent grid (10 tiles per workgroup)."""
    g = torch.Generator(device=DEV).manual_seed(11)
    x = _ints((151552, 896), -2, 2, g)
    w = _ints((896, 896), -2, 2, g, 0.125)
    y, _ = _run(x, w)
    assert torch.equal(y, torch.nn.functional.linear(x, w))


def test_zero_rows_is_a_no_op():
    from verl_amd import _lib as L
    from verl_amd import kernels as K

    w = torch.ones(224, 128, dtype=torch.bfloat16, device=DEV)
    x = torch.ones(1, 128, dtype=torch.bfloat16, device=DEV)
    L.call("va_linear_tn", K._p(x), 128, K._p(w), 128, None, L.VA_BF16, 0, 224, 128, 0, 0, None, 224, K._stream(w))


def test_tile_query_and_argument_checks():
    from verl_amd import _lib as L
    from verl_amd import kernels as K

    lib = L.load()
    assert lib.va_linear_tn_tile(896) == 224 and lib.va_linear_tn_tile(1152) == 192  # the pipelined form's tiles
    assert lib.va_linear_tn_tile(4864) == 256 and lib.va_linear_tn_tile(1000) == 0
    x = torch.zeros(64, 128, dtype=torch.bfloat16, device=DEV)
    w = torch.zeros(224, 128, dtype=torch.bfloat16, device=DEV)
    y = torch.empty(64, 224, dtype=torch.bfloat16, device=DEV)
    s = K._stream(x)
    with pytest.raises(RuntimeError, match="divides N"):
        L.call("va_linear_tn", K._p(x), 128, K._p(w[:200]), 128, None, L.VA_BF16, 64, 200, 128, 0, 0, K._p(y), 224, s)
    with pytest.raises(RuntimeError, match="K %% 64|K % 64"):
        L.call("va_linear_tn", K._p(x), 128, K._p(w), 128, None, L.VA_BF16, 64, 224, 96, 0, 0, K._p(y), 224, s)
    with pytest.raises(RuntimeError, match="aligned"):
        L.call("va_linear_tn", K._p(x[:, 4:]), 128, K._p(w), 128, None, L.VA_BF16, 64, 224, 64, 0, 0, K._p(y), 224, s)
    with pytest.raises(RuntimeError, match="VA_TUNE_LINEAR_TN"):
        L.call("va_set_tuning", L.VA_TUNE_LINEAR_TN, 3)
    with pytest.raises(RuntimeError, match="strides"):
        L.call("va_linear_tn", K._p(x), 64, K._p(w), 128, None, L.VA_BF16, 64, 224, 128, 0, 0, K._p(y), 224, s)
    with pytest.raises(RuntimeError, match="strides"):  # the output's 32-bit buffer offsets
        L.call("va_linear_tn", K._p(x), 128, K._p(w), 128, None, L.VA_BF16, 64, 224, 128, 0, 0, K._p(y), 1 << 22, s)
