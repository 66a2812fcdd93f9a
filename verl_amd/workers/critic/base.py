"""BasePPOCritic — verl/workers/critic/base.py:25-40."""

from abc import ABC, abstractmethod

import torch

from ...protocol import DataProto

__all__ = ["BasePPOCritic"]


class BasePPOCritic(ABC):
    def __init__(self, config):
        super().__init__()
        self.config = config

    @abstractmethod
    def compute_values(self, data: DataProto) -> torch.Tensor:
        """Compute values"""

    @abstractmethod
    def update_critic(self, data: DataProto):
        """Update the critic"""
