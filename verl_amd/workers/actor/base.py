"""Actor plugin interface — mirror of verl/workers/actor/base.py:27-66."""

from abc import ABC, abstractmethod

import torch

from ...protocol import DataProto

__all__ = ["BasePPOActor"]


class BasePPOActor(ABC):
    def __init__(self, config):
        """config: attribute-style dict (omegaconf DictConfig in the reference)."""
        super().__init__()
        self.config = config

    @abstractmethod
    def compute_log_prob(self, data: DataProto) -> torch.Tensor:
        """Per-token log-probs (and entropies) of ``responses`` given input_ids /
        attention_mask / position_ids."""

    @abstractmethod
    def update_policy(self, data: DataProto) -> dict:
        """One PPO update over ``data``; returns a dict of metric lists."""
