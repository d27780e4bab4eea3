"""Synthetic, Oxford-Flowers-shaped image pools generated on the device.

There is no network access for datasets, so benchmarks and smoke tests use a
deterministic pool of smooth random RGB images in [-1, 1] (low-frequency
fields: a coarse random grid bilinearly upsampled plus a few radial "petal"
patterns), resident in HBM.  Training batches are then drawn *on device*
inside the captured step (pool index + cold timestep t from the counter RNG,
pixelation of (x_t, x_{t-1}) in one kernel: ``ops.cold_batch``), replacing the
reference's CPU DataLoader workers (multi_gpu_trainer.py:63-64,
diffusion_loader.py:84-97).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from .. import ops

SITE_DATA = 3
SITE_NOISE = 4


def synthetic_pool(n: int, size=(64, 64), channels: int = 3, seed: int = 0, device="cpu") -> torch.Tensor:
    g = torch.Generator(device="cpu").manual_seed(seed)
    H, W = size
    coarse = torch.rand(n, channels, 6, 6, generator=g) * 2 - 1
    img = F.interpolate(coarse, size=(H, W), mode="bicubic", align_corners=False)
    yy, xx = torch.meshgrid(torch.linspace(-1, 1, H), torch.linspace(-1, 1, W), indexing="ij")
    r = torch.sqrt(xx ** 2 + yy ** 2)
    th = torch.atan2(yy, xx)
    petals = torch.randint(3, 9, (n, 1, 1, 1), generator=g).float()
    phase = torch.rand(n, 1, 1, 1, generator=g) * 2 * math.pi
    radius = 0.4 + 0.4 * torch.rand(n, 1, 1, 1, generator=g)
    flower = torch.sigmoid(12 * (radius * (0.6 + 0.4 * torch.cos(petals * th + phase)) - r))
    color = torch.rand(n, channels, 1, 1, generator=g) * 2 - 1
    img = 0.5 * img + flower * color
    return img.clamp(-1, 1).contiguous().to(device)


class ColdBatcher:
    """Device-side cold-diffusion batch source (graph-capturable).

    Each call draws t ~ U{1..max_t} (and, unless ``idx`` is given, B pool
    indices) from the engine's RNG state and writes (x_t, target, t) into static
    buffers.  target = x_{t-1} (``ColdDownSampleDataset``) or x0 (``target='x0'``,
    ``ColdDownSampleDataset_au``).  With ``idx`` (a static device int64[B] the host
    fills each step from a shard table) the batch follows DistributedSampler order;
    with ``idx_step = (ctr, off)`` as well, ``idx`` is the whole epoch table and the
    batch reads its row ``ctr[0] % rows`` (:func:`ops.stepped_idx`) -- no host copy.
    """

    def __init__(self, pool: torch.Tensor, batch: int, rng: torch.Tensor, max_t: int | None = None,
                 target: str = "prev", idx: torch.Tensor | None = None, idx_step=None):
        self.pool = pool
        B, (C, H, W) = batch, pool.shape[1:]
        self.max_t = max_t or int(math.log2(W))
        dev = pool.device
        self.x_t = torch.empty(B, C, H, W, device=dev)
        self.x_tm1 = torch.empty(B, C, H, W, device=dev)
        self.t = torch.empty(B, dtype=torch.int64, device=dev)
        self.draw = idx is None
        self.idx = torch.empty(B, dtype=torch.int64, device=dev) if idx is None else idx
        self.rng = rng
        self.target = target
        self.idx_step = idx_step

    def fused_spec(self):
        """Deferred form for a consumer that fuses the draw into its patch embedding
        (:func:`ops.patch_embed_cold_fwd`): ``((x_t, target, t), cold)`` without launching
        anything; x_t is not materialised (the patch rows are pixelated from the pool)."""
        cold = (self.pool, SITE_DATA, self.max_t, self.draw, self.target == "x0", self.x_tm1, self.idx, False, 0, 0,
                self.idx_step)
        return (self.x_t, self.x_tm1, self.t), cold

    def __call__(self):
        ops.cold_batch(self.pool, self.rng, SITE_DATA, self.x_t, self.x_tm1, self.t, self.idx, self.max_t,
                       self.draw, idx_step=self.idx_step)
        if self.target == "x0":
            torch.index_select(self.pool, 0, ops.stepped_idx(self.idx, self.idx_step, self.t.shape[0]),
                               out=self.x_tm1)
        return self.x_t, self.x_tm1, self.t


class GaussianBatcher:
    """Device-side Gaussian DDIM batch source: (q_sample(x0, t, eps), x0, t), t ~ U{0..T-1}
    (``DiffusionDataset``, diffusion_loader.py:24-58).  One launch (:func:`ops.gauss_batch`:
    pool draw + noise + q_sample), or none at all when the engine fuses the draw into
    its patch-embedding launch (:meth:`fused_spec`, same values)."""

    def __init__(self, pool: torch.Tensor, batch: int, rng: torch.Tensor, total_steps: int = 2000,
                 idx: torch.Tensor | None = None, idx_step=None):
        self.pool = pool
        B, (C, H, W) = batch, pool.shape[1:]
        dev = pool.device
        self.T = total_steps
        self.x_t = torch.empty(B, C, H, W, device=dev)
        self.x0 = torch.empty(B, C, H, W, device=dev)
        self.t = torch.empty(B, dtype=torch.int64, device=dev)
        self.draw = idx is None
        self.idx = torch.empty(B, dtype=torch.int64, device=dev) if idx is None else idx
        self.rng = rng
        self.B = B
        self.idx_step = idx_step

    def fused_spec(self):
        """``((x_t, x0, t), spec)`` for :func:`ops.patch_embed_cold_fwd` (Gaussian mode)."""
        cold = (self.pool, SITE_DATA, 1, self.draw, True, self.x0, self.idx, False, self.T, SITE_NOISE, self.idx_step)
        return (self.x_t, self.x0, self.t), cold

    def __call__(self):
        ops.gauss_batch(self.pool, self.rng, SITE_DATA, SITE_NOISE, self.T, self.x_t, self.x0, self.t, self.idx,
                        self.draw, idx_step=self.idx_step)
        return self.x_t, self.x0, self.t


def make_batcher(kind: str, pool: torch.Tensor, batch: int, rng: torch.Tensor, total_steps: int = 2000,
                 idx: torch.Tensor | None = None, idx_step=None):
    """Batch source for a dataset kind: 'cold' | 'cold_x0' | 'gaussian' (config key ``dataset``)."""
    if kind == "cold":
        return ColdBatcher(pool, batch, rng, idx=idx, idx_step=idx_step)
    if kind == "cold_x0":
        return ColdBatcher(pool, batch, rng, target="x0", idx=idx, idx_step=idx_step)
    if kind == "gaussian":
        return GaussianBatcher(pool, batch, rng, total_steps, idx=idx, idx_step=idx_step)
    raise ValueError(kind)
