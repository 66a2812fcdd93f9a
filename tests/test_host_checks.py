"""Host-side argument checks and launch planning of the kernel wrappers (no GPU)."""

import numpy as np
import pytest

from verl_amd import kernels as K


@pytest.mark.parametrize("off", [[1, 4, 8], [0, 4, 4, 8], [0, 5, 3, 8], [0], [0, 4, 7]])
def test_seg_offsets_rejects_bad_host_offsets(off):
    """offsets not starting at 0, empty or descending segments, or not ending at the
    row count would make the loss kernels read rows outside [0, B) and divide by zero."""
    with pytest.raises(ValueError, match="seg_off"):
        K.seg_offsets(np.asarray(off), "cpu", rows=8)


def test_own_wgrad_splits_respect_k():
    # H = 896 backbone shapes at the bench's token counts keep their measured plans
    assert K.own_wgrad_splits(896, 896, 151552) == 16
    assert K.own_wgrad_splits(9728, 896, 151552) == 5
    # one 256 x 256 output at 512 tokens (16 K-steps): 2 slices, not 256
    assert K.own_wgrad_splits(256, 256, 512) == 2
    assert K.own_wgrad_splits(256, 256, 32) == 1
    for tokens in (32, 256, 1024, 4096, 65536):
        s = K.own_wgrad_splits(128, 896, tokens)
        assert 1 <= s and (s == 1 or -(-tokens // 32) // s >= K.WGRAD_MIN_STEPS_PER_SLICE)


@pytest.mark.parametrize("lens", [[], [1], [128], [129, 1, 300], [1184, 1100, 1280, 700, 5]])
def test_flash_block_tables(lens):
    """Query blocks (heaviest = latest first) and key blocks (earliest first) of every sequence,
    each (sequence, first row) exactly once, ties broken by sequence."""
    from verl_amd.workers.actor import attention as A

    cu = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    want = [(s, r) for s, n in enumerate(lens) for r in range(0, n, 128)]
    q = [tuple(x) for x in A.flash_block_table(cu).tolist()]
    k = [tuple(x) for x in A.flash_key_block_table(cu).tolist()]
    assert q == sorted(want, key=lambda t: (-t[1], t[0]))
    assert k == sorted(want, key=lambda t: (t[1], t[0]))


@pytest.mark.parametrize("M,N,T", [(9728, 896, 151552), (896, 4864, 151552), (1152, 896, 151552), (896, 896, 151552),
                                   (151936, 896, 131072), (9504, 896, 131072), (200, 136, 1024), (264, 512, 96),
                                   (37888, 3584, 65536), (256, 256, 32)])
@pytest.mark.parametrize("splits", [0, 3])
def test_own_wgrad_plan_mirrors_the_library(M, N, T, splits):
    """kernels.own_wgrad_plan (host mirror of w_plan_tiles) gives the slice count the library plans:
    its workspace query (host code, no GPU) is 4 B x slices x M x N when slices > 1."""
    from verl_amd import _lib as L

    kind, s = K.own_wgrad_plan(M, N, T, splits)
    assert kind in K.WGRAD_TILE_KINDS and 1 <= s
    if splits:
        assert s == splits
    nb = L.load().va_weight_grad_workspace_bytes(T, M, N, splits)
    assert nb == (4 * s * M * N if s > 1 else 0)


def test_own_wgrad_plan_uses_896_dividing_tiles():
    """The bench's backbone and lm_head shapes (H = 896) get tiles with no padded MFMA work."""
    for M, N in [(9728, 896), (896, 4864), (1152, 896), (896, 896), (151936, 896)]:
        kind, s = K.own_wgrad_plan(M, N, 151552 if M < 100000 else 131072)
        tm, tn = K.WGRAD_TILE_KINDS[kind]
        assert (-(-M // tm) * tm) * (-(-N // tn) * tn) <= M * N * 1.01, (M, N, kind)


def test_qkv_rope_rejects_mismatched_operands():
    """va_qkv_rope takes H from x and its rows from the head counts, so the wrappers check
    that the weight, bias and cos / sin tables describe one merged projection (host-side, no GPU)."""
    import torch

    T, H, hq, hk, d = 32, 128, 2, 1, 64
    x = torch.zeros(T, H, dtype=torch.bfloat16)
    w = torch.zeros((hq + 2 * hk) * d, H, dtype=torch.bfloat16)
    b = torch.zeros((hq + 2 * hk) * d, dtype=torch.bfloat16)
    c = torch.zeros(T, d, dtype=torch.bfloat16)
    assert K._qkv_rope_shape_error(x, w, b, c, c, hq, hk, d) is None
    assert "input dimension" in K._qkv_rope_shape_error(x, w[:, :64], b, c, c, hq, hk, d)
    assert "rows" in K._qkv_rope_shape_error(x, w[:-64], b, c, c, hq, hk, d)
    assert "b_all" in K._qkv_rope_shape_error(x, w, b[:-1], c, c, hq, hk, d)
    assert "sin" in K._qkv_rope_shape_error(x, w, b, c, c[:-1], hq, hk, d)
    assert not K.qkv_rope_supported(x, w[:-64], b, c, d, hq, hk, c)
