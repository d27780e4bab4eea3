"""Checkpoint files, byte-compatible with the reference layout.

Reference (multi_gpu_trainer.py:71-80, 94-106, 152-163):

* ``<SavedDir>/<initializing>``    plain ``state_dict`` (init weights shared by all ranks)
* ``<CheckpointDir>/bestloss.pkl``  plain ``state_dict`` (no prefix) of the best val loss
* ``<CheckpointDir>/lastepoch.pkl`` ``{'epoch', 'steps', 'loss_rec', 'metric',
  'state_dict' (DDP: 'module.'-prefixed keys), 'scheduler', 'optimizer'}``

All written with ``torch.save``; optimizer / scheduler entries are standard
``torch.optim.AdamW`` / ``CosineAnnealingLR`` state dicts so files move freely
between this framework and the reference.  Extra keys we add (ignored by the
reference): ``'rng'`` (device RNG seed/step; a resume restores only the
step, each rank keeps its own seed), ``'engine_steps'``, ``'scaler'`` (GradScaler
layout, scale 1: bf16 training needs no loss scaling).

Loading uses ``weights_only=True`` (no arbitrary unpickling).
"""
from __future__ import annotations

import os
from typing import Dict

import torch

PREFIX = "module."


def add_prefix(sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    return {PREFIX + k: v for k, v in sd.items()}


def strip_prefix(sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    if all(k.startswith(PREFIX) for k in sd):
        return {k[len(PREFIX):]: v for k, v in sd.items()}
    return dict(sd)


def cpu_state_dict(model) -> Dict[str, torch.Tensor]:
    return {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}


def _atomic_save(obj, path: str):
    tmp = path + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def save_weights(model, path: str):
    _atomic_save(cpu_state_dict(model), path)


def load_weights(model, path: str, strict: bool = True):
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(sd, dict) and "state_dict" in sd and not any(torch.is_tensor(v) for v in sd.values()):
        sd = sd["state_dict"]
    sd = strip_prefix(sd)
    missing, unexpected = model.load_state_dict(sd, strict=strict)
    eng = getattr(model, "_engine", None)
    if eng is not None:
        eng.sync_params_from_model()
    return missing, unexpected


def save_lastepoch(path: str, model, engine, epoch: int, steps: int, loss_rec: float, metric: float):
    ckpt = {
        "epoch": int(epoch),
        "steps": int(steps),
        "loss_rec": float(loss_rec),
        "metric": float(metric),
        "state_dict": add_prefix(cpu_state_dict(model)),
        "scheduler": engine.scheduler_state_dict(),
        "optimizer": _to_cpu(engine.optimizer_state_dict()),
        "rng": engine.rng.detach().cpu().clone(),
        "engine_steps": int(engine.steps_done),
        # torch.cuda.amp.GradScaler state_dict layout (the reference does not save it,
        # SURVEY §7.4 D15); bf16 needs no loss scaling, so the scale is fixed at 1
        "scaler": {"scale": 1.0, "growth_factor": 2.0, "backoff_factor": 0.5, "growth_interval": 2000,
                   "_growth_tracker": 0},
    }
    _atomic_save(ckpt, path)


def load_lastepoch(path: str, model, engine) -> dict:
    ckpt = torch.load(path, map_location="cpu", weights_only=True)
    model.load_state_dict(strip_prefix(ckpt["state_dict"]), strict=True)
    if engine is not None:
        engine.sync_params_from_model()
        if ckpt.get("optimizer"):
            engine.load_optimizer_state_dict(ckpt["optimizer"])
        if ckpt.get("scheduler"):
            engine.load_scheduler_state_dict(ckpt["scheduler"])
        if ckpt.get("rng") is not None:
            # only the step counter: lastepoch.pkl is written by rank 0, and every
            # rank keeps its own seed (cfg.seed * 1000 + rank) so the ranks' cold
            # timesteps / dropout masks stay independent after a resume
            engine.rng[1:].copy_(ckpt["rng"][1:].to(engine.rng.device))
    return ckpt


def _to_cpu(obj):
    if torch.is_tensor(obj):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return {k: _to_cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_cpu(v) for v in obj)
    return obj
