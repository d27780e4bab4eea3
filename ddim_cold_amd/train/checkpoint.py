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


def lastepoch_dict(snap, epoch: int, steps: int, loss_rec: float, metric: float) -> dict:
    """The reference's ``lastepoch.pkl`` dict (multi_gpu_trainer.py:155-163) from a
    host snapshot of the engine (``TrainEngine.snapshot_to_host``)."""
    snap.wait()
    return {
        "epoch": int(epoch),
        "steps": int(steps),
        "loss_rec": float(loss_rec),
        "metric": float(metric),
        "state_dict": add_prefix(snap.state_dict()),
        "scheduler": snap.scheduler_state_dict(),
        "optimizer": _to_cpu(snap.optimizer_state_dict()),
        "rng": snap.rng.clone(),
        "engine_steps": int(snap.steps_done),
        # torch.cuda.amp.GradScaler state_dict layout (the reference does not save it,
        # SURVEY §7.4 D15); bf16 needs no loss scaling, so the scale is fixed at 1
        "scaler": {"scale": 1.0, "growth_factor": 2.0, "backoff_factor": 0.5, "growth_interval": 2000,
                   "_growth_tracker": 0},
    }


def save_lastepoch(path: str, model, engine, epoch: int, steps: int, loss_rec: float, metric: float):
    """Synchronous ``lastepoch.pkl`` write (the trainer writes through :class:`CheckpointWriter`)."""
    _atomic_save(lastepoch_dict(engine.snapshot_to_host(), epoch, steps, loss_rec, metric), path)


class CheckpointWriter:
    """Epoch-end checkpoints off the training critical path.

    ``submit(take_snapshot, ...)`` returns at once: it first waits for the previous
    write (and re-raises its error), THEN calls ``take_snapshot()``
    (``TrainEngine.snapshot_to_host``: device copies queued on the training stream
    into buffers reused by every snapshot), and a background thread waits for the
    host copy, lays out ``bestloss.pkl`` / ``lastepoch.pkl`` and writes them
    (``torch.save`` to a temp file + atomic rename) while the next epoch trains.
    Taking the snapshot only after the join is what keeps a new snapshot from
    overwriting the buffers a slow previous write is still reading.  An already
    taken snapshot object is accepted too (its caller guarantees no write is in
    flight).  ``join()`` before exit and before anything reads the files."""

    def __init__(self):
        self._thread = None
        self._err: BaseException | None = None
        self.last_write_s = 0.0
        # the last write's phases (s): host copy wait, dict layout, file writes
        self.last_write_parts = (0.0, 0.0, 0.0)

    @staticmethod
    def warm():
        """One-time costs of the first write paid up front, not inside the first
        epoch: torch.save's serializer and the zip writer (to memory)."""
        import io
        buf = io.BytesIO()
        torch.save({"w": torch.zeros(4), "step": 0, "nested": {"a": [1.0]}}, buf)

    def submit(self, snap, lastepoch_path: str, epoch: int, steps: int, loss_rec: float, metric: float,
               best_path: str | None = None):
        import threading
        import time
        self.join()
        if callable(snap) and not hasattr(snap, "wait"):
            snap = snap()  # the snapshot buffers are free: the previous write has finished

        def work():
            try:
                t0 = time.perf_counter()
                snap.wait()
                t1 = time.perf_counter()
                d = lastepoch_dict(snap, epoch, steps, loss_rec, metric)
                t2 = time.perf_counter()
                if best_path is not None:
                    _atomic_save(strip_prefix(d["state_dict"]), best_path)
                _atomic_save(d, lastepoch_path)
                t3 = time.perf_counter()
                self.last_write_s = t3 - t0
                self.last_write_parts = (t1 - t0, t2 - t1, t3 - t2)
            except BaseException as e:  # surfaced by the next join()
                self._err = e

        self._thread = threading.Thread(target=work, name="ckpt-writer", daemon=False)
        self._thread.start()

    def join(self):
        if self._thread is not None:
            self._thread.join()
            self._thread = None
        if self._err is not None:
            e, self._err = self._err, None
            raise RuntimeError(f"checkpoint write failed: {e!r}") from e


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
