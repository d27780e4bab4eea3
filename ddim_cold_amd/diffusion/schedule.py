"""The "sqrt" noise schedule of the reference and DDIM step tables.

* training / q_sample:  abar(t) = 1 - sqrt((t+1)/T)          (diffusion_loader.py:52)
* DDIM update:          abar_t  = 1 - sqrt((t+1)/T) + 1e-5    (ViT.py:232)
                        abar_tk = 1 - sqrt((t+1-k)/T)          (ViT.py:231, no epsilon)
* img2img start noise:  alpha   = 1 - sqrt(t_start/T)          (ViT_draft2drawing.py:395)

The DDIM jump ``k`` must be such that t+1-k >= 0 at the last visited step
(the reference raises ``math domain error`` otherwise); we raise
a clear ``ValueError`` instead.
"""
from __future__ import annotations

import math
from typing import List

import torch


def alpha_bar_train(t, total_steps: int):
    if isinstance(t, torch.Tensor):
        return 1.0 - torch.sqrt((t.double() + 1.0) / total_steps)
    return 1.0 - math.sqrt((t + 1) / total_steps)


def ddim_timesteps(total_steps: int, k: int, start: int | None = None) -> List[int]:
    if k <= 0:
        raise ValueError("DDIM step jump k must be positive")
    start = total_steps - 1 if start is None else start
    ts = list(range(start, 0, -k))
    if not ts:
        raise ValueError("empty DDIM schedule")
    if ts[-1] + 1 - k < 0:
        raise ValueError(
            f"DDIM step jump k={k} incompatible with start={start}, total_steps={total_steps}: the last step "
            f"t={ts[-1]} would need alpha_bar at t+1-k={ts[-1] + 1 - k} < 0 (use k dividing {start + 1})")
    return ts


def ddim_coefficients(total_steps: int, t: int, k: int):
    """(sqrt(a_t), sqrt(1-a_t), sqrt(a_{t-k}), sqrt(1-a_{t-k})) for one DDIM jump."""
    a_t = 1.0 - math.sqrt((t + 1) / total_steps) + 1e-5
    a_tk = 1.0 - math.sqrt((t + 1 - k) / total_steps)
    if a_tk < 0:
        raise ValueError(f"invalid DDIM jump t={t}, k={k}")
    return math.sqrt(a_t), math.sqrt(1.0 - a_t), math.sqrt(a_tk), math.sqrt(1.0 - a_tk)


def ddim_table(total_steps: int, k: int, start: int | None = None, device="cpu"):
    ts = ddim_timesteps(total_steps, k, start)
    coef = torch.tensor([ddim_coefficients(total_steps, t, k) for t in ts], dtype=torch.float32, device=device)
    return ts, coef


def img2img_alpha(t_start: int, total_steps: int) -> float:
    return 1.0 - math.sqrt(t_start / total_steps)


def cold_steps(img_size: int) -> int:
    """Number of cold (de-pixelation) steps = log2(image size) (6 for 64x64, ViT_draft2drawing.py:271)."""
    return int(math.log2(img_size))
