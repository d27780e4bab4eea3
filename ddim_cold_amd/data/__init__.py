"""Data: folder datasets (reference-compatible) and on-device synthetic batch sources."""
from .synthetic import ColdBatcher, GaussianBatcher, synthetic_pool

__all__ = ["ColdBatcher", "GaussianBatcher", "synthetic_pool"]
