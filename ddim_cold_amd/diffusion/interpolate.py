"""Image interpolation through the diffusion latent (the reference's commented-out
experiment, ViT_draft2drawing.py:421-476, made a library function).

For each noise level t_start both images are noised to q(x_t | x0) with
alpha = 1 - sqrt(t_start/T) (independent noise draws, as the reference), the
two noisy images are mixed for every lambda in ``lambdas`` (spherical
interpolation over the whole flattened tensors, or linear), and the mixes are
denoised with DDIM (jump k).  MI355X: every (t_start, lambda) pair of one
k-grid is one batch through :func:`ddim_from_starts` (one hipGraph), instead of
one 11-image batch per noise level.
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch

from .samplers import _unit_host, ddim_from_starts
from .schedule import img2img_alpha


def slerp(a: torch.Tensor, b: torch.Tensor, lam: torch.Tensor) -> torch.Tensor:
    """sin(theta*lam)/sin(theta) * a + sin(theta*(1-lam))/sin(theta) * b,
    theta = angle between flattened a and b (ViT_draft2drawing.py:448-452)."""
    theta = torch.arccos((a.flatten() @ b.flatten()) / (torch.linalg.norm(a) * torch.linalg.norm(b)))
    lam = lam.view(-1, *([1] * (a.dim() - 1))).to(a)
    return (torch.sin(theta * lam) * a + torch.sin(theta * (1 - lam)) * b) / torch.sin(theta)


@torch.no_grad()
def interpolate(model, img1: torch.Tensor, img2: torch.Tensor, t_starts: Sequence[int] = tuple(range(99, 2000, 100)),
                k: int = 10, lambdas: Optional[torch.Tensor] = None, mode: str = "slerp", device=None,
                generator: Optional[torch.Generator] = None, use_graph: bool = True) -> torch.Tensor:
    """Returns CPU images in [0, 1], shape [len(t_starts) + 1, len(lambdas), C, H, W];
    row 0 is the pixel-space linear mix (the reference's first grid row)."""
    device = torch.device(device) if device is not None else next(model.parameters()).device
    T = model.total_steps
    if lambdas is None:
        lambdas = torch.linspace(0, 1, 11)
    n = lambdas.numel()
    img1 = img1.reshape(1, *img1.shape[-3:]).float()
    img2 = img2.reshape(1, *img2.shape[-3:]).float()
    lam = lambdas.view(-1, 1, 1, 1).float()
    rows = [((lam * img2 + (1 - lam) * img1) + 1) / 2]
    # the reference: lambdas1 weights img2 in pixel space and noisy_img1 in slerp
    xs, starts = [], []
    for t0 in t_starts:
        a = img2img_alpha(t0, T)
        n1 = torch.normal(0.0, 1.0, img1.shape, generator=generator) * (1 - a) ** 0.5 + img1 * a ** 0.5
        n2 = torch.normal(0.0, 1.0, img2.shape, generator=generator) * (1 - a) ** 0.5 + img2 * a ** 0.5
        if mode == "slerp":
            mix = slerp(n1, n2, lam.view(-1))
        elif mode == "linear":
            mix = lam * n1 + (1 - lam) * n2
        else:
            raise ValueError(f"mode must be 'slerp' or 'linear', got {mode!r}")
        xs.append(mix)
        starts += [t0] * n
    x = torch.cat(xs)
    top = max(t_starts)
    if all((top - s) % k == 0 for s in t_starts):
        x0 = ddim_from_starts(model, x, starts, k, device, use_graph)
    else:
        x0 = torch.cat([ddim_from_starts(model, x[i * n:(i + 1) * n], starts[i * n:(i + 1) * n], k, device, use_graph)
                        for i in range(len(t_starts))])
    out = _unit_host(x0).view(len(t_starts), n, *img1.shape[-3:])
    return torch.cat([rows[0].unsqueeze(0), out])
