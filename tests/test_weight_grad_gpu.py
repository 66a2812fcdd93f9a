"""va_weight_grad (csrc/wgrad.hip): dW = dY^T X of the backbone's linear layers against an fp32
torch reference, across split-K counts, ragged M / N (clamped columns), strided operands, the
product dispatch (kernels.weight_grad) and run-to-run determinism."""

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _call(dy, x, splits):
    from verl_amd import _lib as L
    from verl_amd import kernels as K

    T, M = dy.shape
    N = x.shape[1]
    out = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=DEV)
    nb = L.load().va_weight_grad_workspace_bytes(T, M, N, splits)
    ws = torch.empty(max(nb // 4, 1), dtype=torch.float32, device=DEV)
    L.call("va_weight_grad", K._p(dy), dy.stride(0), K._p(x), x.stride(0), T, M, N, splits, K._p(ws), ws.numel() * 4,
           K._p(out), K._stream(dy))
    return out


class _tuning:
    """va_set_tuning values for the body of a with-block, restored to the library defaults after."""

    DEFAULTS = {"VA_TUNE_WGRAD_TILES": 4, "VA_TUNE_WGRAD_REMAINDER": 0, "VA_TUNE_WGRAD_MFMA": 32}

    def __init__(self, **kw):
        self.kw = kw

    def __enter__(self):
        from verl_amd import _lib as L

        for k, v in self.kw.items():
            L.call("va_set_tuning", getattr(L, k), v)

    def __exit__(self, *exc):
        from verl_amd import _lib as L

        for k in self.kw:
            L.call("va_set_tuning", getattr(L, k), self.DEFAULTS[k])


def _ref(dy, x):
    return torch.mm(dy.t().float(), x.float())


def _check(got, want):
    scale = want.abs().max().item()
    err = (got.float() - want).abs().max().item()
    assert err <= 8e-3 * scale + 1e-6, (err, scale)


@pytest.mark.parametrize("T,M,N", [(2048, 1152, 896), (4096, 896, 4864), (1024, 200, 136), (96, 264, 512),
                                   (2048, 9728, 896), (1024, 384, 640), (1024, 896, 896)])
@pytest.mark.parametrize("splits", [0, 1, 3, 8])
@pytest.mark.parametrize("tiles,remainder", [(0, 0), (0, 1), (1, 0), (2, 0), (3, 0), (4, 0)])
def test_weight_grad_matches_fp32_reference(T, M, N, splits, tiles, remainder):
    """splits 0 = automatic. VA_TUNE_WGRAD_TILES 0: 256 x 256 tiles, and with VA_TUNE_WGRAD_REMAINDER
    = 1 a dimension that is 128 mod 256 (896, 640, 384) gets 512 x 128 / 128 x 512 remainder tiles
    (explicit splits apply only when there is no remainder); 1 / 2: the cost-model planner's tile
    kinds (256 x 224, 224 x 256, 128 x 448, 448 x 128 for dimensions that are multiples of 224),
    without / with the cross-step fragment pipeline (3: its LDS-DMA spread between the MFMAs; 4: its
    fragment reads too)."""
    g = torch.Generator(device=DEV).manual_seed(T + M + N)
    dy = (torch.randn(T, M, device=DEV, generator=g) * 0.1).to(torch.bfloat16)
    x = torch.randn(T, N, device=DEV, generator=g).to(torch.bfloat16)
    with _tuning(VA_TUNE_WGRAD_TILES=tiles, VA_TUNE_WGRAD_REMAINDER=remainder):
        got = _call(dy, x, splits)
        again = _call(dy, x, splits)
    assert not torch.isnan(got.float()).any()
    _check(got, _ref(dy, x))
    assert torch.equal(got, again)  # deterministic


def test_weight_grad_strided_operands_and_zero_tokens():
    g = torch.Generator(device=DEV).manual_seed(5)
    wide = torch.randn(512, 1024, device=DEV, generator=g).to(torch.bfloat16)
    dy, x = wide[:, :256], wide[:, 512:768]  # row stride 1024, 16-byte aligned column offsets
    _check(_call(dy, x, 2), _ref(dy, x))
    z = _call(dy[:0], x[:0], 1)
    assert torch.equal(z, torch.zeros_like(z))


def test_weight_grad_rejects_bad_shapes():
    from verl_amd import _lib as L

    dy = torch.zeros(100, 64, dtype=torch.bfloat16, device=DEV)  # 100 tokens: not a multiple of 32
    x = torch.zeros(100, 64, dtype=torch.bfloat16, device=DEV)
    with pytest.raises(RuntimeError, match="multiple of 32"):
        _call(dy, x, 1)


def test_product_dispatch_uses_it_and_falls_back():
    """kernels.weight_grad: the own kernel for bf16 [T % 32 == 0] operands (same bits as the direct
    call at the chosen split), hipBLASLt otherwise (T not a multiple of 32)."""
    from verl_amd import kernels as K

    g = torch.Generator(device=DEV).manual_seed(9)
    dy = (torch.randn(4096, 1152, device=DEV, generator=g) * 0.1).to(torch.bfloat16)
    x = torch.randn(4096, 896, device=DEV, generator=g).to(torch.bfloat16)
    got = K.weight_grad(dy, x)
    assert torch.equal(got, _call(dy, x, 0))
    odd = K.weight_grad(dy[:4000], x[:4000])  # hipBLASLt path
    _check(odd, _ref(dy[:4000], x[:4000]))


@pytest.mark.parametrize("T,M,N", [(4096, 9728, 896), (4096, 896, 4864), (2048, 896, 896)])
def test_remainder_tiles_match_full_tiles(T, M, N):
    """VA_TUNE_WGRAD_REMAINDER 0 (256 x 256 tiles throughout) and 1 (remainder tiles) agree to fp32
    summation order: both within the bf16 tolerance of the reference."""
    g = torch.Generator(device=DEV).manual_seed(M + N)
    dy = (torch.randn(T, M, device=DEV, generator=g) * 0.1).to(torch.bfloat16)
    x = torch.randn(T, N, device=DEV, generator=g).to(torch.bfloat16)
    want = _ref(dy, x)
    with _tuning(VA_TUNE_WGRAD_TILES=0):
        full = _call(dy, x, 0)
    with _tuning(VA_TUNE_WGRAD_TILES=0, VA_TUNE_WGRAD_REMAINDER=1):
        rem = _call(dy, x, 0)
    _check(full, want)
    _check(rem, want)


@pytest.mark.parametrize("T,M,N", [(2048, 1152, 896), (4096, 896, 4864), (1024, 200, 136), (96, 264, 512),
                                   (2048, 9728, 896)])
@pytest.mark.parametrize("splits", [0, 1, 3])
@pytest.mark.parametrize("remainder", [0, 1])
def test_weight_grad_16x16x32_form(T, M, N, splits, remainder):
    """VA_TUNE_WGRAD_MFMA = 16 (8 x 4 v_mfma_f32_16x16x32_bf16 blocks per wave, the 8-row image
    swizzle): the fp32 reference's tolerance, deterministic, and on exact-arithmetic operands (small
    integers: every partial sum exact) bitwise equal to the 32x32x16 form."""
    g = torch.Generator(device=DEV).manual_seed(T + M + N + 1)
    dy = (torch.randn(T, M, device=DEV, generator=g) * 0.1).to(torch.bfloat16)
    x = torch.randn(T, N, device=DEV, generator=g).to(torch.bfloat16)
    dyi = torch.randint(-3, 4, (T, M), device=DEV, generator=g).to(torch.bfloat16)
    xi = torch.randint(-3, 4, (T, N), device=DEV, generator=g).to(torch.bfloat16)
    with _tuning(VA_TUNE_WGRAD_TILES=0, VA_TUNE_WGRAD_REMAINDER=remainder, VA_TUNE_WGRAD_MFMA=16):
        got = _call(dy, x, splits)
        again = _call(dy, x, splits)
        exact16 = _call(dyi, xi, splits)
    with _tuning(VA_TUNE_WGRAD_TILES=0, VA_TUNE_WGRAD_REMAINDER=remainder):
        exact32 = _call(dyi, xi, splits)
    assert not torch.isnan(got.float()).any()
    _check(got, _ref(dy, x))
    assert torch.equal(got, again)
    assert torch.equal(exact16, exact32)
    assert torch.equal(exact16.float(), _ref(dyi, xi).to(torch.bfloat16).float())


def test_weight_grad_mfma_setting_is_checked():
    from verl_amd import _lib as L

    with pytest.raises(RuntimeError, match="16 or 32"):
        L.call("va_set_tuning", L.VA_TUNE_WGRAD_MFMA, 8)


@pytest.mark.parametrize("T,M,N", [(2048, 9728, 896), (2048, 896, 4864), (4096, 1152, 896), (4096, 896, 896),
                                   (1024, 9504, 896), (1024, 448, 224), (1024, 200, 136), (512, 3584, 3584)])
@pytest.mark.parametrize("splits", [0, 1, 2, 5])
def test_tile_kinds_bitwise_on_exact_operands(T, M, N, splits):
    """On exact-arithmetic operands (small integers: every partial and slice sum is exact in fp32) the
    planner's tile kinds with and without the fragment pipeline (both DMA placements) give the same bits as the 256 x 256
    tiles of the 32x32x16 form and as the fp32 reference rounded once; on random operands every
    setting meets the reference's tolerance and repeats bitwise."""
    g = torch.Generator(device=DEV).manual_seed(T * 7 + M + N)
    dyi = torch.randint(-3, 4, (T, M), device=DEV, generator=g).to(torch.bfloat16)
    xi = torch.randint(-3, 4, (T, N), device=DEV, generator=g).to(torch.bfloat16)
    dy = (torch.randn(T, M, device=DEV, generator=g) * 0.1).to(torch.bfloat16)
    x = torch.randn(T, N, device=DEV, generator=g).to(torch.bfloat16)
    want = _ref(dy, x)
    exact = {}
    for tiles in (0, 1, 2, 3, 4):
        with _tuning(VA_TUNE_WGRAD_TILES=tiles):
            exact[tiles] = _call(dyi, xi, splits)
            got = _call(dy, x, splits)
            assert torch.equal(got, _call(dy, x, splits))
        _check(got, want)
    assert all(torch.equal(exact[0], exact[t]) for t in (1, 2, 3, 4))
    assert torch.equal(exact[3].float(), _ref(dyi, xi).to(torch.bfloat16).float())


def test_lm_head_weight_gradient_on_the_own_kernel():
    """The lm_head's dW [V, H] = dlogits^T h (V = 151,936 > the backbone's tile cap) goes through
    va_weight_grad in the product dispatch (256 x 224 tiles, K split by the cost model), within the
    fp32 reference's tolerance, with a row stride > V (a [:, :V] view of a padded buffer)."""
    from verl_amd import kernels as K

    T, V, H = 1024, 151936, 896
    g = torch.Generator(device=DEV).manual_seed(11)
    buf = (torch.randn(T, V + 64, device=DEV, generator=g) * 1e-2).to(torch.bfloat16)
    dy = buf[:, :V]
    x = torch.randn(T, H, device=DEV, generator=g).to(torch.bfloat16)
    assert K._OWN_LMHEAD_WGRAD
    got = K.weight_grad(dy, x)
    assert torch.equal(got, _call(dy, x, 0))
    _check(got, _ref(dy, x))


def test_weight_grad_tiles_setting_is_checked():
    from verl_amd import _lib as L

    with pytest.raises(RuntimeError, match="0 .. 4"):
        L.call("va_set_tuning", L.VA_TUNE_WGRAD_TILES, 5)


@pytest.mark.parametrize("kind", [0, 1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("T,M,N", [(1024, 1152, 896), (512, 200, 136), (2048, 896, 4864)])
def test_each_tile_kind_forced(kind, T, M, N):
    """VA_TUNE_WGRAD_KIND forces one tile shape (with the cost model's slice count for it): every kind
    is exact on exact-arithmetic operands and within the reference's tolerance on random ones, also on
    shapes it does not divide (clamped staging, dropped columns)."""
    g = torch.Generator(device=DEV).manual_seed(kind * 101 + T + M + N)
    dyi = torch.randint(-3, 4, (T, M), device=DEV, generator=g).to(torch.bfloat16)
    xi = torch.randint(-3, 4, (T, N), device=DEV, generator=g).to(torch.bfloat16)
    dy = (torch.randn(T, M, device=DEV, generator=g) * 0.1).to(torch.bfloat16)
    x = torch.randn(T, N, device=DEV, generator=g).to(torch.bfloat16)
    from verl_amd import _lib as L

    try:
        L.call("va_set_tuning", L.VA_TUNE_WGRAD_KIND, kind)
        exact = _call(dyi, xi, 0)
        got = _call(dy, x, 0)
    finally:
        L.call("va_set_tuning", L.VA_TUNE_WGRAD_KIND, -1)
    assert torch.equal(exact.float(), _ref(dyi, xi).to(torch.bfloat16).float())
    _check(got, _ref(dy, x))
