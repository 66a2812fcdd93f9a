"""The update RPCs' LR scheduler and perf metrics: closed-form warmup
schedules (torch_functional.py:509-575, built as fsdp_workers.py:425-450 / 1149-1170), the
FlopsCounter's model FLOPs (flops_counter.py:100-132) with an MI355X device entry, and the
update_actor / update_critic wrappers' metric keys and once-per-update scheduler step
(fsdp_workers.py:687-701, 1243-1253). CPU only."""

import math

import pytest
import torch

from verl_amd.utils.config import AttrDict, actor_config, critic_config
from verl_amd.utils.torch_functional import build_lr_scheduler


def _lrs(optim_cfg, n, role="actor", lr=1.0):
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.AdamW([p], lr=lr)
    sch = build_lr_scheduler(opt, AttrDict(optim_cfg), role=role, rank=1)
    out = []
    for _ in range(n):
        out.append(sch.get_last_lr()[0])
        opt.step()
        sch.step()
    return out


def test_constant_warmup_by_steps_and_by_ratio():
    assert _lrs(dict(lr_warmup_steps=3, warmup_style="constant"), 6) == pytest.approx([0, 1 / 3, 2 / 3, 1, 1, 1])
    # negative steps: ratio x total_training_steps (int()), here int(0.25 * 10) = 2
    assert _lrs(dict(lr_warmup_steps=-1, lr_warmup_steps_ratio=0.25, total_training_steps=10), 4) == \
        pytest.approx([0, 0.5, 1, 1])
    # the defaults: no warmup, constant
    assert _lrs(actor_config().optim, 3, lr=1e-6) == pytest.approx([1e-6] * 3)


def test_cosine_warmup_closed_form_actor_and_critic():
    warm, total, mn, cyc = 2, 10, 0.1, 0.5
    want = []
    for s in range(12):
        if s < warm:
            want.append(mn + (1 - mn) * s / warm)
        else:
            prog = (s - warm) / (total - warm)
            want.append(max(mn, math.cos(math.pi * cyc * 2 * prog) * (1 - mn) / 2 + (1 + mn) / 2))
    got = _lrs(dict(lr_warmup_steps=warm, warmup_style="cosine", total_training_steps=total, min_lr_ratio=mn,
                    num_cycles=cyc), 12)
    assert got == pytest.approx(want, abs=1e-12)
    assert got[warm] == pytest.approx(1.0) and got[total] == pytest.approx(mn)
    # the critic's cosine takes neither min_lr_ratio nor num_cycles (fsdp_workers.py:1166-1168)
    crit = _lrs(dict(lr_warmup_steps_ratio=0.2, warmup_style="cosine", total_training_steps=total, min_lr_ratio=mn),
                11, role="critic")
    assert crit[0] == 0.0 and crit[2] == pytest.approx(1.0) and crit[10] == pytest.approx(0.0, abs=1e-12)
    with pytest.raises(NotImplementedError, match="Warmup style linear is not supported"):
        _lrs(dict(warmup_style="linear"), 1)


def test_flops_counter_qwen2_closed_form_and_device_table():
    from verl_amd.utils.flops_counter import FlopsCounter, get_device_flops
    from verl_amd.utils.model import qwen2_config

    cfg = qwen2_config("0.5b")
    h, v, L, ffn, hq, hk, d = 896, 151936, 24, 4864, 14, 2, 64
    dense = (3 * h * ffn + h * (hq * d + 2 * hk * d + hq * d)) * L + 2 * v * h
    seqlens = [1280, 700, 1000]
    want = 6 * dense * sum(seqlens) + 12 * sum(s * s for s in seqlens) * d * hq * L
    est, promised = FlopsCounter(cfg, device_name="AMD Instinct MI355X").estimate_flops(seqlens, 2.0)
    assert est == pytest.approx(want / 2.0 / 1e12, rel=1e-12)
    assert promised == pytest.approx(2500.0)
    assert get_device_flops("T", "AMD Instinct MI300X") == pytest.approx(1336.0)
    assert get_device_flops("P", "AMD Instinct MI350X") == pytest.approx(2.3)
    assert get_device_flops("T", "some GPU") == float("inf")
    assert get_device_flops("T", "AMD Radeon Graphics gfx950:sramecc+:xnack-") == pytest.approx(2500.0)


def test_flops_counter_reads_vl_text_config():
    from verl_amd.utils.flops_counter import FlopsCounter
    from verl_amd.utils.model import qwen2_vl_config

    cfg = qwen2_vl_config("tiny")
    est, _ = FlopsCounter(cfg, device_name="MI355X").estimate_flops([10], 1.0)
    assert cfg.model_type == "qwen2_vl" and est > 0


class _StubActor:
    def __init__(self, opt):
        self.opt = opt

    def update_policy(self, data):
        self.opt.step()  # the update's optimizer step, before the RPC steps the scheduler
        return {"actor/pg_loss": [0.5], "actor/grad_norm": [1.0]}


class _StubCritic:
    def __init__(self, opt):
        self.opt = opt

    def update_critic(self, data):
        self.opt.step()
        return {"critic/vf_loss": [0.25]}


def _batch():
    from verl_amd.protocol import DataProto

    am = torch.ones(4, 10, dtype=torch.int64)
    return DataProto.from_dict(tensors=dict(attention_mask=am), meta_info=dict(global_token_num=[10, 10, 10, 10]))


def test_update_actor_and_critic_rpc_metrics_and_scheduler_steps():
    from verl_amd.utils.flops_counter import FlopsCounter
    from verl_amd.utils.model import qwen2_config
    from verl_amd.workers.dp_workers import ActorWorker, CriticWorker

    acfg = actor_config(ppo_mini_batch_size=2, ppo_micro_batch_size_per_gpu=2,
                        optim=AttrDict(lr=2.0, lr_warmup_steps=2, warmup_style="constant"))
    w = ActorWorker(AttrDict(actor=acfg, rollout=AttrDict(n=1, temperature=1.0)), rollout_n=1)
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.AdamW([p], lr=acfg.optim.lr)
    w.actor = _StubActor(opt)
    w.actor_lr_scheduler = build_lr_scheduler(opt, acfg.optim, rank=1)
    w.flops_counter = FlopsCounter(qwen2_config("tiny"), device_name="MI355X")
    lrs = []
    for _ in range(3):
        m = w.update_actor(_batch()).meta_info["metrics"]
        lrs.append(m["actor/lr"])
        for k in ("perf/mfu/actor", "perf/cpu_memory_used_gb", "actor/pg_loss"):
            assert k in m
        assert m["perf/mfu/actor"] > 0
    assert lrs == pytest.approx([0.0, 1.0, 2.0])

    ccfg = critic_config(ppo_mini_batch_size=2, ppo_micro_batch_size_per_gpu=2,
                         optim=AttrDict(lr=1.0, lr_warmup_steps_ratio=0.5, total_training_steps=4))
    c = CriticWorker(ccfg)
    q = torch.nn.Parameter(torch.zeros(1))
    copt = torch.optim.AdamW([q], lr=1.0)
    c.critic = _StubCritic(copt)
    c.critic_lr_scheduler = build_lr_scheduler(copt, ccfg.optim, role="critic", rank=1)
    c.flops_counter = FlopsCounter(qwen2_config("tiny"), device_name="MI355X")
    got = []
    for _ in range(3):
        m = c.update_critic(_batch()).meta_info["metrics"]
        got.append(m["critic/lr"])
        assert "perf/mfu/critic" in m and m["critic/vf_loss"] == [0.25]
    assert got == pytest.approx([0.0, 0.5, 1.0])


# the reference's own known answers (tests/utils/test_flops_counter.py:30-139: config, two batches of
# sequence lengths, expected TFLOPs at delta_time 1); deepseek_v3 (MLA) is outside this path's families
_FLOPS_KATS = {
    "llama": (dict(model_type="llama", vocab_size=32000, hidden_size=4096, intermediate_size=11008,
                   num_hidden_layers=32, num_attention_heads=32, num_key_value_heads=32),
              (153555818250240 / 1e12, 575955114393600 / 1e12)),
    "qwen2": (dict(model_type="qwen2", vocab_size=152064, hidden_size=3584, intermediate_size=18944,
                   num_hidden_layers=28, num_attention_heads=28, num_key_value_heads=4),
              (170388331954176 / 1e12, 622070178250752 / 1e12)),
    "qwen3": (dict(model_type="qwen3", vocab_size=151936, hidden_size=4096, intermediate_size=12288,
                   num_hidden_layers=36, num_attention_heads=32, num_key_value_heads=8, head_dim=128),
              (185867930959872 / 1e12, 692924253732864 / 1e12)),
    "qwen3_moe": (dict(model_type="qwen3_moe", hidden_size=2048, vocab_size=151936, num_hidden_layers=48,
                       num_key_value_heads=4, num_attention_heads=32, head_dim=128, moe_intermediate_size=768,
                       num_experts_per_tok=8, num_experts=128),
                  (85087060230144 / 1e12, 365944098521088 / 1e12)),
}


@pytest.mark.parametrize("family", sorted(_FLOPS_KATS))
def test_flops_counter_reference_known_answers(family):
    import math
    from types import SimpleNamespace

    from verl_amd.utils.flops_counter import FlopsCounter

    cfg, expected = _FLOPS_KATS[family]
    fc = FlopsCounter(SimpleNamespace(**cfg), device_name="AMD Instinct MI355X")
    for seqlens, want in zip(([512, 1024, 2048], [4096, 4096, 4096]), expected, strict=True):
        got, _ = fc.estimate_flops(seqlens, 1)
        assert math.isclose(got, want), (family, got, want)
