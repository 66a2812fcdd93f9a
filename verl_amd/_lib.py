"""ctypes binding of the C-ABI in ``include/verl_amd.h`` (libverl_amd.so).

This is the only place that loads the native library. The product path has no CPU fallback:
if the library is missing or a tensor is not on a HIP device, the call raises.
"""

from __future__ import annotations

import ctypes
import os
import re
from ctypes import POINTER, c_double, c_float, c_int, c_int64, c_void_p
from pathlib import Path

_PKG = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("VERL_AMD_LIB", _PKG / "lib" / "libverl_amd.so"))
HEADER_PATH = _PKG.parent / "include" / "verl_amd.h"

# constants mirrored from include/verl_amd.h
VA_F32, VA_BF16, VA_F16 = 0, 1, 2
VA_LOGITS_F32 = 256  # va_linear_logprob_fwd dtype flag: fp32 logits (the reference's fused kernel)
VA_MASK_F32, VA_MASK_I64, VA_MASK_I32, VA_MASK_U8 = 0, 1, 2, 3
VA_AGG_TOKEN_MEAN, VA_AGG_SEQ_MEAN_TOKEN_SUM, VA_AGG_SEQ_MEAN_TOKEN_MEAN, VA_AGG_SEQ_MEAN_TOKEN_SUM_NORM = 0, 1, 2, 3
VA_REDUCE_MASKED_SUM, VA_REDUCE_ROW_MASKED_MEAN = 4, 5
VA_KL_NONE, VA_KL_K1, VA_KL_ABS, VA_KL_K2, VA_KL_K3 = -1, 0, 1, 2, 3
VA_ADV_GRPO, VA_ADV_GRPO_NOSTD, VA_ADV_RLOO, VA_ADV_MEAN_ONLY = 0, 1, 2, 3
VA_ADV_OPO, VA_ADV_PASSK, VA_ADV_PASSK_NOSTD = 4, 5, 6
VA_RET_RFPP, VA_RET_REMAX = 0, 1
VA_PL_VANILLA, VA_PL_GPG, VA_PL_CLIP_COV, VA_PL_KL_COV = 0, 1, 2, 3
VA_LOSS_PG, VA_LOSS_CLIPFRAC, VA_LOSS_PPO_KL, VA_LOSS_CLIPFRAC_LOWER = 0, 1, 2, 3
VA_LOSS_KL, VA_LOSS_ENTROPY, VA_LOSS_NTOKENS, VA_LOSS_NROWS, VA_LOSS_NOUT = 4, 5, 6, 7, 8
VA_VLOSS_LOSS, VA_VLOSS_CLIPFRAC, VA_VLOSS_VPRED_MEAN, VA_VLOSS_NTOKENS, VA_VLOSS_NOUT = 0, 1, 2, 3, 4
VA_TUNE_FWD_WAVES_PER_ROW, VA_TUNE_BWD_WAVES_PER_ROW, VA_TUNE_NONTEMPORAL, VA_TUNE_PIPELINE = 1, 2, 3, 4
VA_TUNE_FLASH_GROUPED_DKDV, VA_TUNE_GAE_VARIANT, VA_TUNE_BWD_FLAT, VA_TUNE_SWIGLU_STREAM = 5, 6, 7, 8
VA_TUNE_FLASH_DKDV_QT, VA_TUNE_FLASH_DQ_KB, VA_TUNE_FLASH_FWD_KB, VA_TUNE_GAE_PARTIALS = 9, 10, 11, 12
VA_TUNE_GAE_NT, VA_TUNE_LOSS_VEC = 13, 14
VA_TUNE_WHITEN_SLICE_MIN, VA_TUNE_WHITEN_GRID, VA_TUNE_LINEAR_LOGPROB_TILE = 15, 16, 17
VA_TUNE_WGRAD_REMAINDER, VA_TUNE_FLASH_DMA, VA_TUNE_WGRAD_MFMA, VA_TUNE_WGRAD_TILES = 18, 19, 20, 21
VA_TUNE_ADAMW_MATH, VA_TUNE_WGRAD_KIND, VA_TUNE_LINEAR_TN, VA_TUNE_T256_DEFER = 22, 23, 24, 25
# the library's compiled-in flash-attention staging defaults (csrc/attention.hip), for code that
# changes a setting and restores it
FLASH_TUNING_DEFAULTS = {VA_TUNE_FLASH_DMA: 7, VA_TUNE_FLASH_DQ_KB: 64, VA_TUNE_FLASH_DKDV_QT: 64,
                         VA_TUNE_FLASH_FWD_KB: 64, VA_TUNE_FLASH_GROUPED_DKDV: -1}

ABI_VERSION = 11  # include/verl_amd.h VA_ABI_VERSION

_P = c_void_p
_SIGNATURES: dict[str, tuple] = {
    "va_abi_version": (c_int, []),
    "va_last_error": (ctypes.c_char_p, []),
    "va_device_info": (c_int, [POINTER(c_int), POINTER(c_int), POINTER(c_int)]),
    "va_set_tuning": (c_int, [c_int, c_int]),
    "va_logprob_entropy_fwd": (c_int, [_P, c_int, c_int64, c_int64, c_int64, _P, c_float, _P, _P, _P, _P]),
    "va_logprob_entropy_bwd": (
        c_int,
        [_P, _P, _P, c_int, c_int64, c_int64, c_int64, _P, _P, _P, c_float, _P, c_int64, _P],
    ),
    "va_ppo_loss_workspace_bytes": (c_int64, [c_int64]),
    "va_ppo_loss_fwd": (
        c_int,
        [_P, _P, _P, _P, c_int, _P, _P, c_int64, c_int64, c_float, c_float, c_float, c_int, c_int, c_int, _P,
         c_float, c_int64, _P, c_int64, _P, _P, _P],
    ),
    "va_ppo_loss_bwd": (
        c_int,
        [_P, _P, _P, _P, _P, c_int, _P, c_int64, c_int64, c_float, c_float, c_float, c_int, c_int, c_int, _P,
         c_float, c_int64, _P, c_int64, _P, _P, _P, _P],
    ),
    "va_kl_penalty_fwd": (c_int, [_P, _P, c_int64, c_int, _P, _P]),
    "va_kl_penalty_bwd": (c_int, [_P, _P, _P, c_int64, c_int, _P, _P, _P]),
    "va_agg_workspace_bytes": (c_int64, [c_int64]),
    "va_masked_agg_fwd": (c_int, [_P, _P, c_int, c_int64, c_int64, c_int, _P, _P, _P]),
    "va_masked_agg_bwd": (c_int, [_P, _P, c_int, c_int64, c_int64, c_int, _P, _P, _P]),
    "va_outcome_workspace_bytes": (c_int64, [c_int64]),
    "va_outcome_advantage": (
        c_int,
        [_P, _P, c_int, c_int64, c_int64, _P, _P, c_int64, c_int64, c_float, c_int, _P, _P, _P, _P],
    ),
    "va_row_scores": (c_int, [_P, _P, c_int, c_int64, c_int64, _P, _P, _P]),
    "va_group_coef": (c_int, [_P, _P, _P, _P, c_int64, c_int64, c_float, c_int, _P, _P]),
    "va_broadcast_rows": (c_int, [_P, _P, c_int, c_int64, c_int64, _P, _P]),
    "va_gae_workspace_bytes": (c_int64, [c_int64]),
    "va_gae_partial_count": (c_int64, [c_int64]),
    "va_gae_scan": (c_int, [_P, _P, _P, c_int, c_int64, c_int64, c_float, c_float, _P, _P, _P, _P]),
    "va_masked_row_partials": (c_int, [_P, _P, c_int, c_int64, c_int64, _P, _P]),
    "va_whiten_finalize": (c_int, [_P, c_int64, _P, _P, _P]),
    "va_whiten_apply": (c_int, [_P, _P, _P, c_int, c_int64, c_int64, c_int, _P]),
    "va_gae_advantage_return": (
        c_int,
        [_P, _P, _P, c_int, c_int64, c_int64, c_float, c_float, _P, _P, _P, _P, _P],
    ),
    "va_apply_kl_penalty": (c_int, [_P, _P, _P, _P, c_int, c_int64, c_int64, c_int, c_float, _P, _P, _P]),
    "va_accumulate_grads": (c_int, [c_int, _P, _P, c_int, _P, c_float, _P]),
    "va_adamw_flat": (c_int, [_P, _P, _P, _P, c_int64, c_double, c_double, c_double, c_double, c_double, _P, _P, _P,
                              c_int, _P]),
    "va_rmsnorm_workspace_bytes": (c_int64, [c_int64, c_int64]),
    "va_rmsnorm_fwd": (c_int, [_P, _P, _P, c_int, c_int64, c_int64, c_float, _P, _P, _P, _P]),
    "va_rmsnorm_bwd": (c_int, [_P, _P, _P, _P, _P, c_int, c_int64, c_int64, _P, _P, _P, _P]),
    "va_swiglu_fwd": (c_int, [_P, c_int64, c_int64, c_int, c_int64, c_int64, _P, _P]),
    "va_swiglu_bwd": (c_int, [_P, _P, c_int64, c_int64, c_int, c_int64, c_int64, _P, c_int64, c_int64, _P]),
    "va_gate_up_swiglu": (c_int, [_P, c_int64, _P, c_int64, c_int, c_int64, c_int64, c_int64, c_int, _P, c_int64, _P]),
    "va_gate_up_swiglu_save": (c_int, [_P, c_int64, _P, c_int64, c_int, c_int64, c_int64, c_int64, c_int, _P, c_int64,
                                       _P, c_int64, _P]),
    "va_rope_qkv_fwd": (c_int, [_P, c_int64, _P, _P, c_int, c_int64, c_int64, c_int64, c_int64, _P, _P, _P, _P]),
    "va_value_loss_fwd": (c_int, [_P, _P, _P, _P, c_int, c_int64, c_int64, c_float, c_int, c_int64, _P, c_int64, _P,
                                  _P, _P]),
    "va_value_loss_bwd": (c_int, [_P, _P, _P, _P, _P, c_int, c_int64, c_int64, c_float, c_int, c_int64, _P, c_int64,
                                  _P, _P, _P]),
    "va_discounted_returns": (c_int, [_P, _P, c_int, c_int64, c_int64, c_float, c_int, _P, _P, _P, _P]),
    "va_linear_logprob_workspace_bytes": (c_int64, [c_int64, c_int]),
    "va_linear_logprob_fwd": (
        c_int, [_P, c_int64, _P, c_int64, c_int, _P, c_int64, c_int64, c_int64, c_float, c_int, _P, _P, _P, _P, _P]
    ),
    "va_linear_logprob_bwd": (
        c_int, [_P, c_int64, _P, c_int64, c_int, _P, _P, _P, _P, _P, c_int64, c_int64, c_int64, c_int64, c_int64,
                c_float, c_int, _P, c_int64, _P]
    ),
    "va_flash_attn_fwd": (
        c_int, [_P, _P, _P, _P, _P, c_int64, c_int64, c_int64, c_int64, c_int64, c_int64, c_float, _P, _P, _P]
    ),
    "va_flash_attn_bwd": (
        c_int,
        [_P, _P, _P, _P, _P, _P, _P, _P, c_int64, _P, c_int64, c_int64, c_int64, c_int64, c_int64, c_int64, c_float,
         _P, _P, _P, _P, _P, _P],
    ),
    "va_karmarkar_karp": (c_int, [_P, c_int64, c_int64, c_int, _P, _P]),
    "va_qkv_rope": (c_int, [_P, c_int64, _P, c_int64, _P, _P, _P, c_int, c_int64, c_int64, c_int, c_int, c_int, c_int,
                            _P, _P, _P, _P]),
    "va_rope_qkv_bwd": (c_int, [_P, _P, _P, _P, _P, c_int, c_int64, c_int64, c_int64, c_int64, _P, c_int64, _P]),
    "va_transpose_16": (c_int, [_P, c_int64, c_int64, c_int64, _P, c_int64, _P]),
    "va_linear_tn_tile": (c_int, [c_int64]),
    "va_linear_tn": (c_int, [_P, c_int64, _P, c_int64, _P, c_int, c_int64, c_int64, c_int64, c_int, c_int, _P, c_int64,
                             _P]),
    "va_weight_grad_workspace_bytes": (c_int64, [c_int64, c_int64, c_int64, c_int]),
    "va_column_sum_workspace_bytes": (c_int64, [c_int64, c_int64]),
    "va_column_sum": (c_int, [_P, c_int64, c_int, c_int64, c_int64, _P, c_int64, _P, _P]),
    "va_weight_grad": (c_int, [_P, c_int64, _P, c_int64, c_int64, c_int64, c_int64, c_int, _P, c_int64, _P, _P]),
}

_lib = None


class NativeLibraryError(RuntimeError):
    pass


def header_symbols() -> list[str]:
    """Every function the public header declares (used by the ABI tests)."""
    text = HEADER_PATH.read_text()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char \*)\s*(va_\w+)\s*\(", text, re.M)))


def load():
    """Load libverl_amd.so once and attach the argument types. Raises when it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise NativeLibraryError(
            f"{LIB_PATH} is missing: build the MI355X kernels first "
            "(python -m verl_amd.build, or __graft_entry__.build())"
        )
    lib = ctypes.CDLL(str(LIB_PATH), mode=ctypes.RTLD_GLOBAL)
    # VERL_AMD_LIB_AB=1: an older build loaded for an A/B timing run (tools/f1_ab.py) may lack
    # newer entry points and carry an older ABI version; only what it exports is bound
    ab = os.environ.get("VERL_AMD_LIB_AB") == "1"
    for name, (res, args) in _SIGNATURES.items():
        if ab and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.va_abi_version() != ABI_VERSION and not ab:
        raise NativeLibraryError(f"ABI version mismatch: {lib.va_abi_version()} != {ABI_VERSION}")
    _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = _lib.va_last_error().decode(errors="replace") if _lib is not None else "?"
        raise RuntimeError(f"verl_amd native call {what} failed ({rc}): {msg}")


# va_set_tuning values set through call() in this process (key -> value), for host-side
# heuristics that depend on a kernel choice (e.g. the fused lm_head kernel's vocab split count)
TUNING: dict = {}


def call(name: str, *args) -> None:
    lib = load()
    check(getattr(lib, name)(*args), name)
    if name == "va_set_tuning":
        TUNING[int(args[0])] = int(args[1])


__all__ = ["load", "call", "check", "header_symbols", "LIB_PATH", "NativeLibraryError", "c_double"]
