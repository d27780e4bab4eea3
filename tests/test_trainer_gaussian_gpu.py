"""The trainer on the GPU with the Gaussian DDIM task (DiffusionDataset, diffusion_loader.py:24-58):
graph-captured steps with the q_sample batch drawn inside the patch-embedding launch,
graph-replayed evaluation (one-launch gauss_batch on the fixed validation indices), logs
and checkpoints."""
import dataclasses
import os

import pytest
import torch

from ddim_cold_amd.config import load_config
from ddim_cold_amd.train.trainer import Paths, launch
from ddim_cold_amd.utils.logging import parse_log

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_trainer_gaussian_task_gpu(tmp_path):
    cfg = load_config(os.path.join(ROOT, "configs", "plumbing_gaussian32.yaml")).validate()
    cfg = dataclasses.replace(cfg, image_size=[64, 64], batch_size=16, synthetic_size=256, graph=True,
                              log_every=4, ckpt_dir=str(tmp_path / "Saved_Models"))
    paths = Paths.make(cfg, "gauss64", root=str(tmp_path))
    res = launch(cfg, "gauss64", paths, backend="nccl")
    assert res["steps"] == 256 // 16
    steps, epochs = parse_log(paths.log)
    assert len(epochs) == 1 and 0 < epochs[0][1] < 10  # finite validation loss
    assert all(loss == loss for _, loss, _ in steps)
    last = torch.load(os.path.join(paths.ckpt_dir, "lastepoch.pkl"), weights_only=True)
    temb = last["state_dict"]["module.time_embed.weight"]
    assert temb.shape == (2000, 384) and torch.isfinite(temb).all()
