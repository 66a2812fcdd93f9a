"""Drop-in for the configuration surface of verl/utils/kernel/kernels.py (:47-117): the reduction and
backward-method enums, the module config and set_backward_method, honoured by linear_cross_entropy on the
gfx950 kernels (the reference's Triton kernels themselves are not reproduced: the forward is
va_linear_logprob_fwd, the backward va_linear_logprob_bwd plus hipBLASLt / va_weight_grad GEMMs).

Backward methods (the reference's kernels.py:1380-1553):

* _Split_Dlogits_N (default, as there): dlogits per vocabulary range of 9,504 columns, each range's
  d_hidden (accumulated in fp32) and d_weight GEMMs before the next range;
* _Total_Separate: one range, the whole vocabulary: [N, V] dlogits, then the two GEMMs;
* _Total_Fuse_MN: the reference never writes dlogits and accumulates fp32 d_hidden / d_weight by
  atomic adds from every (row block, vocab block) tile (efficient_entropy_backward_kernel_general_
  mainloop_MN). On MI355X that is ~0.9 MB of fp32 atomics per 256 x 256 tile for each gradient — 557 GB
  per 131,072 x 151,936 pass at the chip's ~1.3 TB/s atomic rate (MI355X_MICROARCH, global float
  atomics), ~0.4 s against ~36 ms for the vocabulary-range path — so this method is served by the
  _Split_Dlogits_N path: the same gradients up to fp32 summation order, the same bounded dlogits memory;
* _Split_Dlogits_M: NotImplementedError, as in the reference.
"""

from __future__ import annotations

from dataclasses import dataclass


@dataclass
class EntropyReductionEnum:
    """kernels.py:47-56; linear_cross_entropy takes the strings "none" / "sum" / "mean"."""

    _None = 0
    _Sum = 1
    _Mean = 2


def get_entropy_reduction_enum_number(reduction: str) -> int:
    """kernels.py:59-70."""
    _enum = EntropyReductionEnum._None
    if reduction == "none":
        _enum = EntropyReductionEnum._None
    elif reduction == "sum":
        _enum = EntropyReductionEnum._Sum
    elif reduction == "mean":
        _enum = EntropyReductionEnum._Mean
    else:
        raise ValueError(f"Invalid reduction: {reduction}")
    return _enum


def get_entropy_reduction_enum(ce_reduction: int) -> int:
    """kernels.py:73-86."""
    if ce_reduction not in (EntropyReductionEnum._None, EntropyReductionEnum._Sum, EntropyReductionEnum._Mean):
        raise ValueError(f"Invalid ce_reduction: {ce_reduction}")
    return ce_reduction


@dataclass
class BackwardEnum:
    """kernels.py:89-100 (the same values)."""

    _Total_Fuse_MN = 0
    _Total_Separate = 1
    _Split_Dlogits_N = 2
    _Split_Dlogits_M = 3


@dataclass
class Config:
    """kernels.py:103-107 (_use_triton: kept for the interface; the kernels here are HIP)."""

    _backward: int = BackwardEnum._Split_Dlogits_N
    _use_triton: bool = True


_config = Config()


def set_backward_method(backward_method: int):
    """kernels.py:112-117."""
    if backward_method not in (BackwardEnum._Total_Fuse_MN, BackwardEnum._Total_Separate,
                               BackwardEnum._Split_Dlogits_N, BackwardEnum._Split_Dlogits_M):
        raise ValueError(f"Invalid backward method: {backward_method}")
    _config._backward = backward_method


def backward_vocab_per_split(vocab: int, default: int) -> int:
    """The dlogits range width linear_cross_entropy's backward uses under the configured method."""
    if _config._backward == BackwardEnum._Split_Dlogits_M:
        raise NotImplementedError("BackwardEnum._Split_Dlogits_M is not implemented yet")
    if _config._backward == BackwardEnum._Total_Separate:
        return max(vocab, 8)
    return default
