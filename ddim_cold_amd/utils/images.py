"""Image grid writing (PNG via PIL) and the fixed ``get_next_path``.

Reference: the sampling CLI plots grids with matplotlib ImageGrid
(``ViT.py:284-305``) and names files with ``get_next_path`` whose loop never
increments its counter (``ViT.py:307-313``).  Grids here are
assembled as tensors and written with PIL (no plotting dependency).
"""
from __future__ import annotations

import os
from typing import Sequence

import numpy as np
import torch


def get_next_path(pth: str) -> str:
    """First non-existing path among pth, <stem>_1<ext>, <stem>_2<ext>, ..."""
    stem, ext = os.path.splitext(pth)
    i, path = 1, pth
    while os.path.isfile(path):
        path = f"{stem}_{i}{ext}"
        i += 1
    return path


def make_grid(images: torch.Tensor, nrow: int, pad: int = 2, value: float = 1.0) -> torch.Tensor:
    """[N, C, H, W] in [0, 1] -> [C, rows*(H+pad)+pad, nrow*(W+pad)+pad]."""
    images = images.detach().float().cpu().clamp(0, 1)
    N, C, H, W = images.shape
    ncol = min(nrow, N)
    nrows = (N + nrow - 1) // nrow
    grid = torch.full((C, nrows * (H + pad) + pad, ncol * (W + pad) + pad), value)
    for i in range(N):
        r, c = divmod(i, nrow)
        y, x = pad + r * (H + pad), pad + c * (W + pad)
        grid[:, y:y + H, x:x + W] = images[i]
    return grid


def save_image(img: torch.Tensor, path: str, scale: int = 1):
    from PIL import Image
    arr = (img.detach().float().cpu().clamp(0, 1) * 255).round().byte().permute(1, 2, 0).numpy()
    if arr.shape[2] == 1:
        arr = arr[:, :, 0]
    im = Image.fromarray(np.ascontiguousarray(arr))
    if scale != 1:
        im = im.resize((im.width * scale, im.height * scale), Image.NEAREST)
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    im.save(path)
    return path


def save_grid(images: torch.Tensor, path: str, nrow: int, scale: int = 2) -> str:
    return save_image(make_grid(images, nrow), path, scale)


def save_sequence_grid(seq: Sequence[torch.Tensor], path: str, scale: int = 2) -> str:
    """Trajectory grid: one row per sample, one column per recorded step (``ViT.py:285-294``)."""
    st = torch.stack(list(seq), dim=0).transpose(0, 1)  # [N, steps, C, H, W]
    N, S = st.shape[:2]
    return save_grid(st.flatten(0, 1), path, nrow=S, scale=scale)
