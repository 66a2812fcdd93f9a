"""Actor workers: BasePPOActor (plugin interface) and DataParallelPPOActor (MI355X DP actor)."""

from .base import BasePPOActor
from .dp_actor import DataParallelPPOActor

__all__ = ["BasePPOActor", "DataParallelPPOActor"]
