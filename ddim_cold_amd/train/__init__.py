"""Training runtime: fused engine, trainer, checkpoints, logging."""
from .engine import EngineConfig, TrainEngine

__all__ = ["EngineConfig", "TrainEngine"]
