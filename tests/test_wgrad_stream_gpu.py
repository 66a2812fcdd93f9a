"""Backbone weight gradients on a side stream (workers/grad_sync.MixedPrecisionParams
.enable_wgrad_stream, kernels._MergedLinear): the bench's actor configuration (packed micro-batches,
fused backbone, flash attention, bf16 weights + fp32 masters) trains bitwise like the single-stream
backward over two mini-batch updates with gradient accumulation, and the side stream is really used."""

import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _worker(side: bool, model="tiny", seed=5):
    from verl_amd.utils.config import AttrDict, actor_config
    from verl_amd.utils.model import build_qwen2
    from verl_amd.workers.dp_workers import ActorWorker

    cfg = AttrDict(
        actor=actor_config(ppo_mini_batch_size=4, ppo_micro_batch_size_per_gpu=8, use_kl_loss=True,
                           kl_loss_coef=0.01, kl_loss_type="low_var_kl", grad_clip=1.0, loss_agg_mode="token-mean",
                           pack_pad_multiple=256, logprob_inplace_backward=False, wgrad_side_stream=side,
                           optim=AttrDict(lr=1e-3, weight_decay=0.01, betas=(0.9, 0.999))),
        rollout=AttrDict(log_prob_micro_batch_size_per_gpu=8, temperature=1.0))
    w = ActorWorker(cfg, rollout_n=4)
    w.init_model(build_qwen2(model, device=DEV, seed=seed))
    return w


def _batch(seed=3):
    from verl_amd.utils.synthetic import make_grpo_batch

    b = make_grpo_batch(n_prompts=8, n=4, prompt_len=48, response_len=96, vocab=4096, min_prompt=5,
                        dense_responses=False, min_response=9, seed=seed).to(DEV)
    g = torch.Generator(device=DEV).manual_seed(seed)
    lp = -torch.rand(b.batch["responses"].shape, device=DEV, generator=g)
    b.batch["old_log_probs"] = lp + 0.05 * torch.randn(lp.shape, device=DEV, generator=g)
    b.batch["ref_log_prob"] = lp + 0.1 * torch.randn(lp.shape, device=DEV, generator=g)
    return b


def _params(worker):
    return torch.cat([p.detach().float().reshape(-1) for p in worker.actor.grad_reducer.masters])


def test_side_stream_weight_grads_bitwise():
    from verl_amd.trainer.ppo.core_algos import AdvantageEstimator

    ws = {side: _worker(side) for side in (False, True)}
    assert ws[True].actor.wgrad_side_stream and not ws[False].actor.wgrad_side_stream
    metrics = {}
    for side, w in ws.items():
        for step in range(2):
            b = _batch(seed=3 + step)
            w.compute_advantage(b, AdvantageEstimator.GRPO, norm_adv_by_std_in_grpo=True)
            out = w.update_actor(b)
        metrics[side] = out.meta_info["metrics"]
    torch.cuda.synchronize()
    assert ws[True].actor.grad_reducer.side_stream_grads > 0
    assert ws[False].actor.grad_reducer.side_stream_grads == 0
    assert torch.equal(_params(ws[False]), _params(ws[True]))
    for a, b in zip(ws[False].module.parameters(), ws[True].module.parameters()):
        assert torch.equal(a, b)
    for k in ("actor/pg_loss", "actor/grad_norm"):
        assert metrics[False][k] == metrics[True][k], k
