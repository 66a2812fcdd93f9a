"""Host-side drop-ins of verl/utils/torch_functional.py: the WSD schedule (:641-694), padding
helpers (:307-328, :407-419), get_unpad_data (:629-638) and compute_grad_norm (:249-254), against
values worked out from the reference source."""

import math

import pytest
import torch

from verl_amd.utils import torch_functional as vF


def test_wsd_schedule_phases():
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=1.0)
    sch = vF.get_wsd_schedule_with_warmup(opt, num_warmup_steps=10, num_training_steps=110, min_lr_ratio=0.1,
                                          stable_ratio=0.9)
    lrs = []
    for _ in range(115):
        lrs.append(opt.param_groups[0]["lr"])
        opt.step()
        sch.step()
    # remaining 100: 90 stable, 10 decay
    assert lrs[0] == 0.0 and lrs[5] == pytest.approx(0.5) and lrs[10] == 1.0 and lrs[99] == 1.0
    assert lrs[100] == pytest.approx(1.0)  # decay progress 0: cos(0) -> 1
    assert lrs[105] == pytest.approx(0.9 * 0.5 * (1 + math.cos(math.pi * 0.5)) + 0.1)
    assert lrs[110] == pytest.approx(0.1) and lrs[114] == pytest.approx(0.1)


def test_padding_helpers_and_unpad_data():
    ids = torch.tensor([[0, 0, 5, 6], [1, 2, 3, 4]])
    am = torch.tensor([[0, 0, 1, 1], [1, 1, 1, 1]])
    assert vF.remove_pad_token(ids, am) == [[5, 6], [1, 2, 3, 4]]
    t = torch.tensor([[1, 2], [3, 4]])
    assert vF.pad_sequence_to_length(t, 4, -1).tolist() == [[1, 2, -1, -1], [3, 4, -1, -1]]
    assert vF.pad_sequence_to_length(t, 4, -1, left_pad=True).tolist() == [[-1, -1, 1, 2], [-1, -1, 3, 4]]
    assert vF.pad_sequence_to_length(t, 1, -1) is t
    assert vF.pad_2d_list_to_length([[1], [2, 3]], 0).tolist() == [[1, 0], [2, 3]]
    assert vF.pad_2d_list_to_length([[1], [2, 3]], 0, max_length=3).tolist() == [[1, 0, 0], [2, 3, 0]]
    idx, cu, mx = vF.get_unpad_data(am)
    assert idx.tolist() == [2, 3, 4, 5, 6, 7] and cu.tolist() == [0, 2, 6] and cu.dtype == torch.int32 and mx == 4


def test_compute_grad_norm_is_the_sum_of_squares():
    m = torch.nn.Linear(3, 2)
    m.weight.grad = torch.tensor([[1.0, 2.0, 0.0], [0.0, 0.0, 2.0]])
    m.bias.grad = None
    assert vF.compute_grad_norm(m) == pytest.approx(9.0)  # 1 + 4 + 4, no square root
    m.bias.grad = torch.tensor([3.0, 0.0])
    assert vF.compute_grad_norm(m) == pytest.approx(18.0)
