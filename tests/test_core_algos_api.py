"""The core_algos / ray_trainer mirror keeps the reference's plugin API and error surface
(tests/trainer/ppo/test_core_algos_on_cpu.py:29-131). Host logic only: CPU."""

import unittest
from enum import Enum

import numpy as np
import pytest
import torch

import verl_amd.trainer.ppo.core_algos as core_algos
from verl_amd.protocol import DataProto
from verl_amd.trainer.ppo import ray_trainer
from verl_amd.trainer.ppo.core_algos import get_adv_estimator_fn, register_adv_est
from verl_amd.utils.config import AttrDict


def mock_test_fn():
    pass


class TestRegisterAdvEst(unittest.TestCase):
    def setUp(self):
        self._saved = dict(core_algos.ADV_ESTIMATOR_REGISTRY)
        core_algos.ADV_ESTIMATOR_REGISTRY.clear()
        core_algos.ADV_ESTIMATOR_REGISTRY.update({"gae": lambda x: x * 2, "vtrace": lambda x: x + 1})
        self.reg = core_algos.ADV_ESTIMATOR_REGISTRY

    def tearDown(self):
        core_algos.ADV_ESTIMATOR_REGISTRY.clear()
        core_algos.ADV_ESTIMATOR_REGISTRY.update(self._saved)

    def test_register_new_function(self):
        @register_adv_est("test_estimator")
        def fn():
            pass

        self.assertIs(self.reg["test_estimator"], fn)

    def test_register_with_enum(self):
        class E(Enum):
            TEST = "test_enum_estimator"

        @register_adv_est(E.TEST)
        def fn():
            pass

        self.assertIs(self.reg["test_enum_estimator"], fn)

    def test_duplicate_same_function_ok(self):
        register_adv_est("dup")(mock_test_fn)
        register_adv_est("dup")(mock_test_fn)
        self.assertIs(self.reg["dup"], mock_test_fn)

    def test_duplicate_different_function_raises(self):
        @register_adv_est("conflict")
        def f1():
            pass

        with self.assertRaises(ValueError):

            @register_adv_est("conflict")
            def f2():
                pass

    def test_get_valid_and_invalid(self):
        assert get_adv_estimator_fn("gae")(5) == 10
        assert get_adv_estimator_fn("vtrace")(5) == 6
        with pytest.raises(ValueError) as e:
            get_adv_estimator_fn("invalid_name")
        assert "Unknown advantage estimator simply: invalid_name" in str(e.value)
        with pytest.raises(ValueError):
            get_adv_estimator_fn("GAE")


def test_builtin_registry_contents():
    names = {e.value for e in core_algos.AdvantageEstimator}
    assert names <= set(core_algos.ADV_ESTIMATOR_REGISTRY)
    assert core_algos.get_adv_estimator_fn(core_algos.AdvantageEstimator.GRPO) is core_algos.compute_grpo_outcome_advantage
    assert set(core_algos.POLICY_LOSS_REGISTRY) == {"gpg", "clip_cov", "kl_cov"}
    with pytest.raises(ValueError, match="Unsupported loss mode: nope"):
        core_algos.get_policy_loss_fn("nope")


def test_kl_controllers():
    c = core_algos.get_kl_controller(AttrDict(type="adaptive", kl_coef=0.1, target_kl=0.05, horizon=100))
    c.update(current_kl=0.2, n_steps=10)  # error clipped to +0.2
    assert abs(c.value - 0.1 * (1 + 0.2 * 10 / 100)) < 1e-12
    f = core_algos.get_kl_controller(AttrDict(type="fixed", kl_coef=0.3))
    f.update(1.0, 5)
    assert f.value == 0.3
    with pytest.raises(AssertionError):
        core_algos.get_kl_controller(AttrDict(type="adaptive", kl_coef=0.1, target_kl=0.05, horizon=0))
    with pytest.raises(NotImplementedError):
        core_algos.get_kl_controller(AttrDict(type="other"))


def test_error_surface_before_device():
    x = torch.zeros(2, 3)
    with pytest.raises(ValueError, match="Invalid loss_agg_mode: bogus"):
        core_algos.agg_loss(x, x, "bogus")
    with pytest.raises(NotImplementedError):
        core_algos.kl_penalty(x, x, "full")
    with pytest.raises(AssertionError, match="clip_ratio_c"):
        core_algos.compute_policy_loss(x, x, x, x, cliprange=0.2, clip_ratio_c=1.0)
    with pytest.raises(ValueError, match="Invalid loss_agg_mode"):
        core_algos.compute_policy_loss(x, x, x, x, cliprange=0.2, loss_agg_mode="bad")


def test_compute_advantage_dispatches_by_module_attribute(monkeypatch):
    """ray_trainer.py:247, 266 call core_algos.<fn> by attribute: replacing it is honoured."""
    calls = []

    def fake_grpo(token_level_rewards, response_mask, index, norm_adv_by_std_in_grpo=True, **kw):
        calls.append(("grpo", norm_adv_by_std_in_grpo, list(index)))
        return token_level_rewards + 1, token_level_rewards + 2

    def fake_gae(token_level_rewards, values, response_mask, gamma, lam):
        calls.append(("gae", gamma, lam))
        return values, values

    monkeypatch.setattr(core_algos, "compute_grpo_outcome_advantage", fake_grpo)
    monkeypatch.setattr(core_algos, "compute_gae_advantage_return", fake_gae)
    d = DataProto.from_dict(
        tensors={"token_level_rewards": torch.zeros(2, 3), "responses": torch.zeros(2, 3),
                 "attention_mask": torch.ones(2, 5), "values": torch.ones(2, 3)},
        non_tensors={"uid": ["a", "a"]},
    )
    ray_trainer.compute_advantage(d, core_algos.AdvantageEstimator.GRPO, norm_adv_by_std_in_grpo=False)
    assert calls[-1] == ("grpo", False, ["a", "a"])
    assert torch.equal(d.batch["advantages"], torch.ones(2, 3))
    assert torch.equal(d.batch["response_mask"], torch.ones(2, 3))  # attention_mask[:, -R:]
    ray_trainer.compute_advantage(d, core_algos.AdvantageEstimator.GAE, gamma=0.9, lam=0.8)
    assert calls[-1] == ("gae", 0.9, 0.8)


def test_compute_advantage_other_estimators_use_registry(monkeypatch):
    seen = {}

    def fake(token_level_rewards, response_mask, config=None, index=None, **kw):
        seen.update(index=None if index is None else list(index), config=config)
        return token_level_rewards, token_level_rewards

    monkeypatch.setitem(core_algos.ADV_ESTIMATOR_REGISTRY, "rloo", fake)
    d = DataProto.from_dict(tensors={"token_level_rewards": torch.zeros(2, 3), "response_mask": torch.ones(2, 3)},
                            non_tensors={"uid": np.array(["x", "y"], dtype=object)})
    ray_trainer.compute_advantage(d, "rloo", config={"k": 1})
    assert seen["index"] == ["x", "y"] and seen["config"] == {"k": 1}
