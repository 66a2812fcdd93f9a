"""PPOTrainerStep / RayPPOTrainer orchestration on CPU with recording workers: the reference's
fit() step order (ray_trainer.py:1195-1330), critic warmup gating, in-reward KL only when
configured, metric reduction (utils/metric/utils.py:23-56)."""

import numpy as np
import pytest
import torch

from oracle import reference_ops as ref
from verl_amd.protocol import DataProto
from verl_amd.utils.config import AttrDict


class _Actor:
    def __init__(self, log, ref_policy=False):
        self.log = log
        self.ref_policy = object() if ref_policy else None

    def compute_log_prob(self, data):
        self.log.append("old_log_prob")
        B, R = data.batch["responses"].shape
        return DataProto.from_dict(tensors={"old_log_probs": -torch.ones(B, R), "entropys": torch.full((B, R), 2.0)})

    def compute_ref_log_prob(self, data):
        self.log.append("ref_log_prob")
        return DataProto.from_dict(tensors={"ref_log_prob": -torch.ones_like(data.batch["old_log_probs"])})

    def compute_advantage(self, data, est, **kw):
        self.log.append(f"advantage:{est.value}")
        assert "token_level_rewards" in data.batch.keys()
        data.batch["advantages"] = data.batch["token_level_rewards"].clone()
        data.batch["returns"] = data.batch["token_level_rewards"].clone()
        return data

    def update_actor(self, data):
        self.log.append("update_actor")
        assert "advantages" in data.batch.keys() and "old_log_probs" in data.batch.keys()
        return DataProto(meta_info={"metrics": {"actor/pg_loss": [1.0, 3.0], "actor/grad_norm_max": [2.0, 5.0]}})


class _Critic:
    def __init__(self, log):
        self.log = log

    def compute_values(self, data):
        self.log.append("values")
        return DataProto.from_dict(tensors={"values": torch.zeros_like(data.batch["old_log_probs"])})

    def update_critic(self, data):
        self.log.append("update_critic")
        return DataProto(meta_info={"metrics": {"critic/vf_loss": [0.5]}})


def _batch(B=4, P=3, R=5):
    ids = torch.randint(0, 10, (B, P + R))
    am = torch.ones(B, P + R, dtype=torch.long)
    return DataProto.from_dict(
        tensors=dict(input_ids=ids, attention_mask=am, position_ids=torch.arange(P + R).expand(B, -1).clone(),
                     responses=ids[:, P:].clone(), token_level_scores=torch.ones(B, R)),
        non_tensors=dict(uid=np.array(["a", "a", "b", "b"], dtype=object)))


def _cfg(est, warmup=0):
    return AttrDict(algorithm=AttrDict(adv_estimator=est, gamma=1.0, lam=1.0, norm_adv_by_std_in_grpo=True,
                                       use_kl_in_reward=False, kl_penalty="kl"),
                    actor_rollout_ref=AttrDict(actor=AttrDict(loss_agg_mode="token-mean"), rollout=AttrDict(n=2)),
                    trainer=AttrDict(critic_warmup=warmup))


@pytest.fixture(autouse=True)
def _cpu_agg(monkeypatch):
    from verl_amd.trainer.ppo import trainer_step

    monkeypatch.setattr(trainer_step.core_algos, "agg_loss", ref.agg_loss)


def test_step_order_gae_with_critic_and_ref():
    from verl_amd.trainer.ppo.trainer_step import PPOTrainerStep

    log = []
    step = PPOTrainerStep(_cfg("gae"), _Actor(log, ref_policy=True), critic=_Critic(log), device=torch.device("cpu"))
    batch, met = step.step(_batch())
    assert log == ["old_log_prob", "ref_log_prob", "values", "advantage:gae", "update_critic", "update_actor"]
    assert "response_mask" in batch.batch.keys() and batch.meta_info["global_token_num"] == [8] * 4
    assert met["actor/entropy"] == pytest.approx(2.0)
    assert met["actor/pg_loss"] == pytest.approx(2.0) and met["actor/grad_norm_max"] == 5.0
    assert met["critic/vf_loss"] == 0.5


def test_critic_warmup_skips_actor_update_and_grpo_needs_no_critic():
    from verl_amd.trainer.ppo.trainer_step import PPOTrainerStep

    # fit() numbers steps from 1 (ray_trainer.py:1099, 1118) and updates the actor once
    # critic_warmup <= global_steps (:1315): warmup 2 skips step 1 only, warmup 1 skips nothing
    log = []
    step = PPOTrainerStep(_cfg("gae", warmup=2), _Actor(log), critic=_Critic(log), device=torch.device("cpu"))
    step.step(_batch())
    assert "update_actor" not in log and log[-1] == "update_critic"
    log.clear()
    step.step(_batch())
    assert log[-1] == "update_actor"
    log.clear()
    one = PPOTrainerStep(_cfg("gae", warmup=1), _Actor(log), critic=_Critic(log), device=torch.device("cpu"))
    one.step(_batch())
    assert log[-2:] == ["update_critic", "update_actor"]
    log2 = []
    g = PPOTrainerStep(_cfg("grpo"), _Actor(log2), device=torch.device("cpu"))
    g.step(_batch())
    assert log2 == ["old_log_prob", "advantage:grpo", "update_actor"]
    with pytest.raises(ValueError):
        PPOTrainerStep(_cfg("gae"), _Actor([]), device=torch.device("cpu"))


def test_ray_trainer_surface_builds_workers_from_the_role_mapping():
    from verl_amd.trainer.ppo.ray_trainer import RayPPOTrainer
    from verl_amd.trainer.ppo.trainer_step import Role

    log = []
    actor = _Actor(log, ref_policy=True)
    tr = RayPPOTrainer(_cfg("grpo"), tokenizer=None,
                       role_worker_mapping={Role.ActorRollout: lambda: actor, Role.RefPolicy: lambda: None})
    tr.init_workers()
    tr.step_runner.device = torch.device("cpu")
    mets = tr.fit([_batch(), _batch()])
    assert len(mets) == 2 and tr.global_steps == 3  # steps 1 and 2 ran
    assert [m["training/global_step"] for m in mets] == [1, 2]
    assert log.count("ref_log_prob") == 2 and log.count("update_actor") == 2


def test_reduce_metrics_matches_reference_rules():
    from verl_amd.trainer.ppo.trainer_step import reduce_metrics

    out = reduce_metrics({"loss": [1.0, 2.0, 3.0], "max_reward": [5.0, 8.0, 6.0], "min_error": [0.1, 0.05, 0.2]})
    assert out == {"loss": 2.0, "max_reward": 8.0, "min_error": 0.05}


def test_attention_mask_host_copy_reuse_and_invalidation():
    """The update reuses the host copy of the attention mask that compute_log_prob took in the same
    step (no second D2H drain), and never a stale one: an in-place change or another tensor
    invalidates it, and refresh=True always copies."""
    from types import SimpleNamespace

    from verl_amd.workers.actor.dp_actor import DataParallelPPOActor

    me = SimpleNamespace(_am_cache=None)
    am = torch.ones(4, 6, dtype=torch.int64)
    a1 = DataParallelPPOActor._mask_host(me, am, refresh=True)
    assert DataParallelPPOActor._mask_host(me, am, refresh=False) is a1  # reused
    am[0, 0] = 0  # in place: version bump
    a2 = DataParallelPPOActor._mask_host(me, am, refresh=False)
    assert a2 is not a1 and a2[0, 0] == 0
    other = torch.zeros(4, 6, dtype=torch.int64)
    a3 = DataParallelPPOActor._mask_host(me, other, refresh=False)
    assert a3 is not a2 and a3.sum() == 0
    assert DataParallelPPOActor._mask_host(me, other, refresh=True) is not a3  # refresh copies


def test_attention_mask_host_mirror_is_used_until_the_device_tensor_is_written():
    """DataProto.to(cuda) keeps a private host clone of the mask it moved (protocol.HOST_MIRRORED_KEY);
    _mask_host plans from it instead of a device->host copy, but not once the device tensor was
    written in place. Writes to the caller's host tensor after the move (through numpy views or a
    reused loader buffer, which bump no version) cannot reach the clone. Emulated on host
    tensors: the mirror attribute is what .to sets."""
    from types import SimpleNamespace

    from verl_amd.protocol import HOST_MIRRORED_KEY, DataProto
    from verl_amd.workers.actor.dp_actor import DataParallelPPOActor

    me = SimpleNamespace(_am_cache=None)
    src = torch.ones(3, 5, dtype=torch.int64)
    dev = torch.ones(3, 5, dtype=torch.int64)  # stands in for the device copy
    mirror = src.clone()
    dev._va_host_mirror = (mirror, dev._version)
    got = DataParallelPPOActor._mask_host(me, dev)
    assert np.shares_memory(got, mirror.numpy())  # the mirror itself, no copy
    src.numpy()[1, 1] = 0  # the caller's buffer reused after the move: the clone still holds the moved mask
    me._am_cache = None
    got = DataParallelPPOActor._mask_host(me, dev)
    assert got[1, 1] == 1
    me._am_cache = None
    dev[0, 0] = 0  # the device side changed: the mirror is stale
    got = DataParallelPPOActor._mask_host(me, dev)
    assert not np.shares_memory(got, mirror.numpy()) and got[0, 0] == 0
    # DataProto.to only mirrors a host -> device move, and then as a clone
    d = DataProto.from_dict({HOST_MIRRORED_KEY: torch.ones(2, 4, dtype=torch.int64)})
    d.to("cpu")
    assert getattr(d.batch[HOST_MIRRORED_KEY], "_va_host_mirror", None) is None


def test_device_metrics_mapping_and_callbacks(capsys):
    """dp_actor.DeviceMetrics (the update's metrics, read back asynchronously): tensor and host
    values in list order, scalars kept, keys set before the first read kept, on_ready callbacks
    run once after the values are in, and the non-finite grad_norm warning."""
    from verl_amd.workers.actor.dp_actor import DeviceMetrics

    m = DeviceMetrics({"actor/pg_loss": [torch.tensor(0.5), 0.25, torch.tensor([1.5])],
                       "actor/grad_norm": [torch.tensor(float("inf"))], "actor/kl_coef": [0.001], "perf/x": 3.0})
    m["actor/lr"] = 1e-6
    seen = []
    m.add_on_ready(lambda mm: seen.append(mm["actor/pg_loss"][0]))
    m.add_on_ready(lambda mm: mm.__setitem__("perf/mfu/actor", 0.4))
    assert m["actor/pg_loss"] == [0.5, 0.25, 1.5] and m["perf/x"] == 3.0 and m["actor/lr"] == 1e-6
    assert seen == [0.5] and m["perf/mfu/actor"] == 0.4
    assert set(m) == {"actor/pg_loss", "actor/grad_norm", "actor/kl_coef", "perf/x", "actor/lr", "perf/mfu/actor"}
    assert "not finite" in capsys.readouterr().out
    m.add_on_ready(lambda mm: seen.append(1))  # already resolved: runs at once
    assert seen == [0.5, 1] and dict(m)["actor/kl_coef"] == [0.001]
    import pickle

    back = pickle.loads(pickle.dumps(m))
    assert type(back) is dict and back == dict(m)


def test_fused_kernel_impl_backend_selects_the_logits_precision():
    """actor_rollout_ref.model.fused_kernel_options.impl_backend (ppo_trainer.yaml:91-94): "torch" (the
    default) is FusedLinearForPPO's bf16 logits, "triton" the Triton kernel's fp32 logits
    (fsdp_workers.py:298-309); an explicit fused_kernel_fp32_logits wins."""
    from verl_amd.utils.config import actor_config
    from verl_amd.utils.model import build_qwen2
    from verl_amd.workers.actor import DataParallelPPOActor

    m = build_qwen2("tiny", device="cpu")
    for kw, want in (({}, False), ({"fused_kernel_options": {"impl_backend": "torch"}}, False),
                     ({"fused_kernel_options": {"impl_backend": "triton"}}, True),
                     ({"fused_kernel_options": {"impl_backend": "triton"}, "fused_kernel_fp32_logits": False}, False)):
        a = DataParallelPPOActor(actor_config(**kw), m, torch.optim.SGD(m.parameters(), lr=0.0))
        assert a.fused_kernel_fp32_logits is want, kw
