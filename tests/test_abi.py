"""The C-ABI library loads, exports every symbol include/verl_amd.h declares, and the product path
refuses CPU tensors (no CPU fallback). No compute calls: this runs without a GPU."""

import ctypes

import numpy as np
import pytest
import torch

from verl_amd import _lib as L


@pytest.fixture(scope="module")
def lib():
    if not L.LIB_PATH.exists():
        from verl_amd import build

        build.build()
    return L.load()


def test_header_declares_the_expected_entry_points():
    syms = L.header_symbols()
    for s in ["va_logprob_entropy_fwd", "va_logprob_entropy_bwd", "va_ppo_loss_fwd", "va_ppo_loss_bwd",
              "va_outcome_advantage", "va_gae_advantage_return", "va_whiten_finalize", "va_kl_penalty_fwd"]:
        assert s in syms
    assert len(syms) == len(L._SIGNATURES)


def test_library_exports_every_header_symbol(lib):
    raw = ctypes.CDLL(str(L.LIB_PATH))
    missing = [s for s in L.header_symbols() if not hasattr(raw, s)]
    assert not missing, missing
    assert set(L.header_symbols()) == set(L._SIGNATURES)


def test_abi_version_and_workspace_queries(lib):
    assert lib.va_abi_version() == 11
    assert lib.va_ppo_loss_workspace_bytes(10) == 8 * (2 * 10 * 8 + 8)
    assert lib.va_agg_workspace_bytes(10) == 8 * (2 * 10 * 8 + 8)
    assert lib.va_gae_workspace_bytes(7) == 8 * (6 * 7 + 8)
    assert lib.va_gae_partial_count(7) == 7 and lib.va_gae_partial_count(8192) == 8192
    try:
        assert lib.va_set_tuning(L.VA_TUNE_GAE_PARTIALS, 4) == 0
        assert lib.va_gae_partial_count(7) == 2 and lib.va_gae_partial_count(8192) == 2048
        assert lib.va_set_tuning(L.VA_TUNE_GAE_PARTIALS, 3) == -1
    finally:
        lib.va_set_tuning(L.VA_TUNE_GAE_PARTIALS, 0)


def test_argument_validation_without_device(lib):
    # invalid shapes are rejected before any HIP call
    rc = lib.va_logprob_entropy_fwd(None, 1, 4, 0, 0, None, 1.0, None, None, None, None)
    assert rc == -1 and b"vocab" in lib.va_last_error()
    rc = lib.va_ppo_loss_fwd(None, None, None, None, 0, None, None, 0, 5, 0.8, 1.2, 3.0, 0, -1, 0, None, 0.0, 0,
                             None, 0, None, None, None)
    assert rc == -1 and b"empty batch" in lib.va_last_error()
    # the clip_cov / kl_cov modes need their token selection
    rc = lib.va_ppo_loss_fwd(1, 1, 1, 1, 0, None, None, 2, 5, 0.8, 1.2, 3.0, 0, -1, L.VA_PL_CLIP_COV, None, 0.0, 0,
                             None, 0, 1, 1, None)
    assert rc == -1 and b"selection" in lib.va_last_error()
    # loss micro-batch segments: negative seg_rows, or offsets with n_seg outside [1, B]
    rc = lib.va_ppo_loss_fwd(1, 1, 1, 1, 0, None, None, 2, 5, 0.8, 1.2, 3.0, 0, -1, 0, None, 0.0, -1, None, 0, 1, 1,
                             None)
    assert rc == -1 and b"bad segments" in lib.va_last_error()
    rc = lib.va_value_loss_fwd(1, 1, 1, 1, 0, 2, 5, 0.5, 0, 0, 1, 3, 1, 1, None)
    assert rc == -1 and b"bad segments" in lib.va_last_error()
    assert lib.va_outcome_workspace_bytes(10) == 4 * 3 * 10
    # weight gradient: tokens not a multiple of 32
    rc = lib.va_weight_grad(1, 64, 1, 64, 100, 64, 64, 1, None, 0, 1, None)
    assert rc == -1 and b"multiple of 32" in lib.va_last_error()
    # the launch's own plan needs more workspace than the caller passed
    rc = lib.va_weight_grad(16, 64, 16, 32, 4096, 64, 32, 3, 16, 4 * 3 * 64 * 32 - 4, 16, None)
    assert rc == -1 and b"workspace bytes" in lib.va_last_error()
    assert lib.va_weight_grad_workspace_bytes(4096, 64, 32, 3) == 4 * 3 * 64 * 32
    rc = lib.va_group_coef(1, None, 1, 1, 4, 8, 1e-6, L.VA_ADV_OPO, 1, None)
    assert rc == -1 and b"lengths" in lib.va_last_error()
    assert lib.va_logprob_entropy_fwd(None, 1, 0, 10, 10, None, 1.0, None, None, None, None) == 0  # n_rows 0: no-op
    # fused lm_head backward: V % 4 != 0 is an argument error; N = 0 is a no-op
    rc = lib.va_linear_logprob_bwd(None, 64, None, 64, L.VA_BF16, None, None, None, None, None, 4, 64, 130, 0, 130,
                                   1.0, 1, None, 130, None)
    assert rc == -1 and b"V % 4" in lib.va_last_error()
    assert lib.va_linear_logprob_bwd(None, 64, None, 64, L.VA_BF16, None, None, None, None, None, 0, 64, 128, 0, 128,
                                     1.0, 1, None, 128, None) == 0
    # vocab ranges (ABI 6): inside [0, V), a multiple of 4 wide (V itself need not be)
    rc = lib.va_linear_logprob_bwd(None, 64, None, 64, L.VA_BF16, None, None, None, None, None, 4, 64, 128, 64, 132,
                                   1.0, 1, None, 68, None)
    assert rc == -1 and b"vocab range" in lib.va_last_error()
    assert lib.va_linear_logprob_bwd(None, 64, None, 64, L.VA_BF16, None, None, None, None, None, 0, 64, 130, 2, 130,
                                     1.0, 1, None, 128, None) == 0


def test_product_path_rejects_cpu_tensors():
    from verl_amd import kernels as K
    from verl_amd.trainer.ppo import core_algos

    x = torch.randn(2, 5)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        K.logprob_entropy(x, torch.zeros(2, dtype=torch.long))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        core_algos.compute_policy_loss(x, x, x, torch.ones(2, 5), cliprange=0.2)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        core_algos.compute_grpo_outcome_advantage(x, torch.ones(2, 5), np.array([0, 0]))


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    monkeypatch.setattr(L, "_lib", None)
    monkeypatch.setattr(L, "LIB_PATH", tmp_path / "nope.so")
    with pytest.raises(L.NativeLibraryError, match="missing"):
        L.load()


def test_header_constants_match_the_python_mirror():
    """Every #define VA_* value in include/verl_amd.h equals the constant _lib.py mirrors."""
    import re

    text = L.HEADER_PATH.read_text()
    defs = dict(re.findall(r"^#define (VA_[A-Z0-9_]+) \(?(-?\d+)\)?", text, re.M))
    mirrored = {k: v for k, v in vars(L).items() if k.startswith("VA_") and isinstance(v, int)}
    assert mirrored, "no constants mirrored"
    for name, value in mirrored.items():
        assert name in defs, name
        assert int(defs[name]) == value, (name, defs[name], value)
    for key in ("VA_TUNE_GAE_VARIANT", "VA_TUNE_BWD_FLAT", "VA_TUNE_SWIGLU_STREAM"):
        assert key in mirrored


def test_tuning_keys_without_device(lib):
    for key in (L.VA_TUNE_GAE_VARIANT, L.VA_TUNE_BWD_FLAT, L.VA_TUNE_SWIGLU_STREAM):
        assert lib.va_set_tuning(key, 0) == 0
    assert lib.va_set_tuning(L.VA_TUNE_GAE_VARIANT, 0) == 0
    assert lib.va_set_tuning(L.VA_TUNE_BWD_FLAT, -1) == 0
    assert lib.va_set_tuning(L.VA_TUNE_SWIGLU_STREAM, -1) == 0
    for key, val in L.FLASH_TUNING_DEFAULTS.items():  # the attention staging keys, at their defaults
        assert lib.va_set_tuning(key, val) == 0, key
    assert lib.va_set_tuning(L.VA_TUNE_FLASH_DQ_KB, 96) == -1
    assert lib.va_set_tuning(99, 1) == -1


def test_gate_up_swiglu_save_validation_without_device(lib):
    # ABI 8: the projection buffer is required and must hold 2F columns
    rc = lib.va_gate_up_swiglu_save(1, 64, 1, 64, L.VA_BF16, 4, 64, 128, 1, 1, 128, None, 256, None)
    assert rc == -1 and b"null projection" in lib.va_last_error()
    rc = lib.va_gate_up_swiglu_save(16, 64, 16, 64, L.VA_BF16, 4, 64, 128, 1, 16, 128, 16, 200, None)
    assert rc == -1 and b"2F" in lib.va_last_error()
    assert lib.va_gate_up_swiglu_save(None, 64, None, 64, L.VA_BF16, 0, 64, 128, 1, None, 128, None, 256, None) == 0


def test_transpose_validation_without_device(lib):
    rc = lib.va_transpose_16(None, 8, 7, 8, None, 8, None)
    assert rc == -1 and b"multiples of 8" in lib.va_last_error()
    rc = lib.va_transpose_16(None, 8, 16, 16, None, 16, None)
    assert rc == -1 and b"strides" in lib.va_last_error()
    assert lib.va_transpose_16(None, 8, 0, 8, None, 8, None) == 0  # empty: no-op
