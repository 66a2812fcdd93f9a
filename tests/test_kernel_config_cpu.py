"""verl_amd.utils.kernel.kernels: the reference's configuration surface of its fused lm_head kernels
(verl/utils/kernel/kernels.py:47-117) — enum values, reduction mapping, set_backward_method and the
dlogits range width each backward method gives linear_cross_entropy."""

import pytest

from verl_amd.utils.kernel import kernels as KK


def test_enum_values_match_the_reference():
    assert (KK.BackwardEnum._Total_Fuse_MN, KK.BackwardEnum._Total_Separate, KK.BackwardEnum._Split_Dlogits_N,
            KK.BackwardEnum._Split_Dlogits_M) == (0, 1, 2, 3)
    assert (KK.EntropyReductionEnum._None, KK.EntropyReductionEnum._Sum, KK.EntropyReductionEnum._Mean) == (0, 1, 2)
    assert [KK.get_entropy_reduction_enum_number(r) for r in ("none", "sum", "mean")] == [0, 1, 2]
    with pytest.raises(ValueError):
        KK.get_entropy_reduction_enum_number("max")
    assert KK.get_entropy_reduction_enum(2) == 2
    with pytest.raises(ValueError):
        KK.get_entropy_reduction_enum(5)
    assert KK.Config()._backward == KK.BackwardEnum._Split_Dlogits_N


def test_backward_method_selects_the_range_width():
    try:
        assert KK.backward_vocab_per_split(151936, 9504) == 9504
        KK.set_backward_method(KK.BackwardEnum._Total_Separate)
        assert KK.backward_vocab_per_split(151936, 9504) == 151936
        KK.set_backward_method(KK.BackwardEnum._Total_Fuse_MN)  # served by the vocabulary-range path
        assert KK.backward_vocab_per_split(151936, 9504) == 9504
        KK.set_backward_method(KK.BackwardEnum._Split_Dlogits_M)
        with pytest.raises(NotImplementedError):
            KK.backward_vocab_per_split(151936, 9504)
        with pytest.raises(ValueError):
            KK.set_backward_method(7)
    finally:
        KK.set_backward_method(KK.BackwardEnum._Split_Dlogits_N)
