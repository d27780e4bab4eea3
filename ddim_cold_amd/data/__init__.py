"""Data: reference-compatible folder datasets, an on-device image cache and
graph-capturable on-device batch sources (synthetic or cached)."""
from .datasets import (ColdDownSampleDataset, ColdDownSampleDataset_au, DATASETS, DeviceImageCache, DiffusionDataset,
                       list_images, load_image, pil_loader, shard_indices)
from .synthetic import ColdBatcher, GaussianBatcher, make_batcher, synthetic_pool

__all__ = ["ColdDownSampleDataset", "ColdDownSampleDataset_au", "DATASETS", "DeviceImageCache", "DiffusionDataset",
           "list_images", "load_image", "pil_loader", "shard_indices", "ColdBatcher", "GaussianBatcher",
           "make_batcher", "synthetic_pool"]
