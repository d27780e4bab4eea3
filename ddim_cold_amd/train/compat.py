"""The reference trainer's library interface (L5), on the MI355X runtime.

``multi_gpu_trainer.py`` of the reference exposes three functions besides its
``__main__`` block:

* ``printLog(string, fileName)``                     (multi_gpu_trainer.py:18-23)
* ``init_process_group(world_size, rank)``           (multi_gpu_trainer.py:25-30)
* ``evaluate(model, dataloader, device)``            (multi_gpu_trainer.py:32-45)
* ``main(rank, world_size, initializing, amp, batch_size, epoch_num, lr, resume,
  datadir, SavedDir, log, CheckpointDir, image_size, diff_step, patch_size,
  embed_dim, depth, head)``                          (multi_gpu_trainer.py:47-165)

Same signatures and semantics here.  ``evaluate`` takes any iterable of
``(x_t, target, t)`` batches (a torch ``DataLoader`` over ``ColdDownSampleDataset``
in the reference) and runs the fused forward; the per-batch losses are summed on
the device with one host sync at the end instead of a ``.item()`` per batch.
``main`` maps its arguments onto an :class:`ExperimentConfig` and runs
:func:`trainer.train_worker` (device-resident data, replayed step graphs, the
reference's log lines and checkpoint files).
"""
from __future__ import annotations

import math
import os
from typing import Iterable, List, Optional, Sequence

import torch
import torch.nn.functional as F

from ..utils.logging import printLog  # noqa: F401  (re-exported: the reference's printLog)

REFERENCE_ADDR = "127.0.0.1"
REFERENCE_PORT = 16666  # multi_gpu_trainer.py:28 tcp://127.0.0.1:16666


def init_process_group(world_size: int, rank: int, backend: Optional[str] = None) -> bool:
    """``dist.init_process_group`` over TCP to 127.0.0.1 (multi_gpu_trainer.py:25-30):
    'nccl' (RCCL over xGMI) on GPUs, 'gloo' on the CPU.  The port is the reference's
    16666 unless MASTER_PORT is set (so two jobs can share a host)."""
    from ..parallel import dist as pdist
    os.environ.setdefault("MASTER_ADDR", REFERENCE_ADDR)
    os.environ.setdefault("MASTER_PORT", str(REFERENCE_PORT))
    if world_size <= 1:
        return pdist.init_single(backend=backend, device_index=rank)
    return pdist.init_distributed(backend=backend, rank=rank, world_size=world_size)


@torch.no_grad()
def evaluate(model, dataloader: Iterable, device) -> float:
    """Mean over batches of the per-batch smooth-L1 loss in eval mode
    (multi_gpu_trainer.py:32-45).  ``model``: a DiffusionVisionTransformer or a
    wrapper holding one as ``.module`` (DDP style); batches ``(x_t, target, t)``.
    Returns NaN for an empty loader (numpy's mean of no values)."""
    net = getattr(model, "module", model)
    net.eval()
    dev = torch.device(device)
    total = torch.zeros((), dtype=torch.float64, device=dev)
    n = 0
    for noisy_img, img, t in dataloader:
        noisy_img = noisy_img.to(dev, non_blocking=True)
        img = img.to(dev, non_blocking=True)
        t = t.to(dev, non_blocking=True)
        out = net(noisy_img, t)
        total += F.smooth_l1_loss(out.float(), img.float()).double()
        n += 1
    if n == 0:
        return math.nan
    return float(total.item()) / n


def config_from_args(world_size: int, initializing: str, amp: bool, batch_size: int, epoch_num: Sequence[int],
                     lr: float, resume: str, datadir: Sequence[str], image_size: Sequence[int], diff_step: int,
                     patch_size: int, embed_dim: int, depth: int, head: int, **extra):
    """:class:`ExperimentConfig` for the reference worker's arguments.  ``batch_size``
    is the per-GPU batch the worker receives (already doubled for AMP by the
    reference launcher, multi_gpu_trainer.py:191-194) and ``lr`` the final learning
    rate (multi_gpu_trainer.py:196): the config's derived values reproduce both."""
    from ..config import ExperimentConfig
    batch_size = int(batch_size)
    cfg = ExperimentConfig(initializing=os.path.basename(initializing), resume=resume or "none", AMP=False,
                           num_gpus=int(world_size), batch_size=batch_size, epoch=[int(e) for e in epoch_num],
                           base_lr=float(lr) * 512.0 / (batch_size * int(world_size)),
                           dataStorage=[str(d) for d in datadir], image_size=[int(v) for v in image_size],
                           diff_step=int(diff_step), patch_size=int(patch_size), embed_dim=int(embed_dim),
                           depth=int(depth), head=int(head), **extra)
    return cfg.validate()  # ``amp``: bf16 compute needs no loss scaling (checkpoints keep a scale-1 scaler)


def main(rank: int, world_size: int, initializing: str, amp: bool, batch_size: int, epoch_num: List[int], lr: float,
         resume: str, datadir: Sequence[str], SavedDir: str, log: str, CheckpointDir: str, image_size: Sequence[int],
         diff_step: int, patch_size: int, embed_dim: int, depth: int, head: int, backend: Optional[str] = None,
         **extra) -> dict:
    """The reference worker ``main(rank, world_size, initializing, amp, batch_size,
    epoch_num, lr, resume, datadir, SavedDir, log, CheckpointDir, image_size,
    diff_step, patch_size, embed_dim, depth, head)`` (multi_gpu_trainer.py:47-165):
    one rank of the data-parallel run -- process group, shared init weights under
    ``SavedDir + initializing``, the ``Date`` / ``TrainSet batchs`` / ``steps:`` /
    ``epoch:`` lines in ``log``, ``bestloss.pkl`` / ``lastepoch.pkl`` under
    ``CheckpointDir`` and ``resume`` -- on :func:`trainer.train_worker`.  ``extra``:
    optional :class:`ExperimentConfig` extension keys (e.g. ``synthetic=True``).
    Returns the worker's result dict (steps, loss_rec, best_loss, history, ...)."""
    from .trainer import Paths, train_worker
    cfg = config_from_args(world_size, initializing, amp, batch_size, epoch_num, lr, resume, datadir, image_size,
                           diff_step, patch_size, embed_dim, depth, head, **extra)
    saved = SavedDir if SavedDir.endswith("/") else SavedDir + "/"
    os.makedirs(saved, exist_ok=True)
    os.makedirs(CheckpointDir, exist_ok=True)
    paths = Paths(saved_dir=saved, ckpt_dir=CheckpointDir if CheckpointDir.endswith("/") else CheckpointDir + "/",
                  log=log)
    if world_size > 1 and "MASTER_PORT" not in os.environ:
        os.environ["MASTER_ADDR"] = os.environ.get("MASTER_ADDR", REFERENCE_ADDR)
        os.environ["MASTER_PORT"] = str(REFERENCE_PORT)
    return train_worker(int(rank), int(world_size), cfg, os.path.basename(os.path.normpath(CheckpointDir)), paths,
                        backend=backend)
