"""Text log + scalar writer with the reference's formats.

Reference: ``printLog`` (multi_gpu_trainer.py:18-23) appends one line per call;
line formats kept so existing log parsers work:

* ``Date: <asctime>``, ``TrainSet batchs:<n>``, ``TestSet batchs:<n>``   (:83-85)
* ``steps: %8d loss: %.4f time_cost: %.2f``                              (:137)
* ``epoch: %4d    loss: %.5f    time:<asctime>``                          (:150)
* ``resuming from epoch %8d of <path>``, ``recovering best_loss %4f``      (:99, :106)

Extra (our) lines are prefixed ``# `` so they do not collide with the
reference regexes.  TensorBoard is optional (``SummaryWriter`` when
importable, rank 0 only — the reference constructed one on every rank);
otherwise scalars go to ``scalars.csv`` next to the log.
"""
from __future__ import annotations

import os
import re
import time


def printLog(string: str, fileName: str):
    with open(fileName, "a") as f:
        f.write(string + "\n")
    return 0


def asctime() -> str:
    return time.asctime(time.localtime(time.time()))


def fmt_steps(steps: int, loss: float, time_cost: float) -> str:
    return f"steps: {steps:8d} loss: {loss:.4f} time_cost: {time_cost:.2f}"


def fmt_epoch(epoch: int, loss: float) -> str:
    return f"epoch: {epoch:4d}    loss: {loss:.5f}    time:{asctime()}"


STEPS_RE = re.compile(r"steps:\s+(\d+) loss: ([\d.]+) time_cost: ([\d.]+)")
EPOCH_RE = re.compile(r"epoch:\s+(\d+)\s+loss: ([\d.]+)")


def parse_log(path: str):
    """Parse a (reference or ours) train.log -> (steps list, epochs list)."""
    steps, epochs = [], []
    with open(path) as f:
        for line in f:
            m = STEPS_RE.search(line)
            if m:
                steps.append((int(m.group(1)), float(m.group(2)), float(m.group(3))))
                continue
            m = EPOCH_RE.search(line)
            if m:
                epochs.append((int(m.group(1)), float(m.group(2))))
    return steps, epochs


class ScalarWriter:
    def __init__(self, logdir: str, enabled: bool = True):
        self.enabled = enabled
        self.tb = None
        self.csv = None
        if not enabled:
            return
        try:
            from torch.utils.tensorboard import SummaryWriter  # noqa: F401
            self.tb = SummaryWriter(log_dir=os.path.join(logdir, "runs"))
        except Exception:
            os.makedirs(logdir, exist_ok=True)
            self.csv = os.path.join(logdir, "scalars.csv")

    def add_scalar(self, tag: str, value: float, step: int):
        if not self.enabled:
            return
        if self.tb is not None:
            self.tb.add_scalar(tag, value, step)
        elif self.csv is not None:
            with open(self.csv, "a") as f:
                f.write(f"{tag},{step},{value}\n")

    def close(self):
        if self.tb is not None:
            self.tb.close()
