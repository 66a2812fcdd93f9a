"""a14, dp_actor.py:272-288: an update whose clipped-gradient norm is not finite is skipped
(parameters, optimizer moments and step counts untouched), a warning names the rank, and the next
update trains normally. The fused AdamW skips the step on the device (found_inf), so the update
has no host sync; a non-fused optimizer takes the reference's host check."""

import numpy as np
import pytest
import torch


pytestmark = pytest.mark.gpu


def _actor(device, fused):
    from verl_amd.utils.config import actor_config
    from verl_amd.utils.model import build_qwen2
    from verl_amd.workers.actor import DataParallelPPOActor
    from verl_amd.workers.dp_workers import make_param_manager

    model = build_qwen2("tiny", device=device, seed=3, attn_implementation="sdpa")
    mgr = make_param_manager(model, bucket_mb=1, mixed_precision=True, zero=False)
    opt = torch.optim.AdamW(mgr.optimizer_params(), lr=1e-3, fused=fused)
    cfg = actor_config(ppo_mini_batch_size=4, ppo_micro_batch_size_per_gpu=2, grad_clip=1.0)
    return model, opt, DataParallelPPOActor(cfg, model, opt, grad_reducer=mgr)


def _batch(device, poison: bool):
    from verl_amd.utils.synthetic import make_grpo_batch

    data = make_grpo_batch(n_prompts=1, n=4, prompt_len=8, response_len=12, vocab=4096, min_prompt=2,
                           dense_responses=False, min_response=3, seed=4, device=device)
    b = data.batch
    g = torch.Generator(device=device).manual_seed(5)
    b["old_log_probs"] = -8.0 - torch.rand(b["responses"].shape, device=device, generator=g)
    b["advantages"] = torch.randn(b["responses"].shape, device=device, generator=g) * b["response_mask"]
    if poison:
        b["advantages"][0, 0] = float("nan")
    data.meta_info["temperature"] = 1.0
    return data


def _run(device, capsys, fused):
    model, opt, actor = _actor(device, fused)
    masters = [p.detach().clone() for p in opt.param_groups[0]["params"]]
    weights = [p.detach().clone() for p in model.parameters()]
    met = actor.update_policy(_batch(device, poison=True))
    assert not np.isfinite(met["actor/grad_norm"][0])
    assert "not finite" in capsys.readouterr().out
    for a, b in zip(opt.param_groups[0]["params"], masters, strict=True):
        assert torch.equal(a.detach(), b)
    for a, b in zip(model.parameters(), weights, strict=True):
        assert torch.equal(a.detach(), b)
    for st in opt.state.values():
        assert float(st["step"]) == 0.0
        assert torch.count_nonzero(st["exp_avg"]) == 0 and torch.count_nonzero(st["exp_avg_sq"]) == 0
    met = actor.update_policy(_batch(device, poison=False))
    assert np.isfinite(met["actor/grad_norm"][0]) and met["actor/grad_norm"][0] > 0
    assert any(not torch.equal(a.detach(), b) for a, b in zip(model.parameters(), weights, strict=True))
    assert all(float(st["step"]) == 1.0 for st in opt.state.values())


@pytest.mark.parametrize("fused", [True, False])
def test_nonfinite_update_skipped(capsys, fused):
    _run("cuda", capsys, fused)
