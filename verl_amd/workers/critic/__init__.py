from .base import BasePPOCritic
from .dp_critic import DataParallelPPOCritic

__all__ = ["BasePPOCritic", "DataParallelPPOCritic"]
