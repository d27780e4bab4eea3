"""Plain eager PyTorch DDIM sampler — the sampling comparator named in BASELINE.md.

The reference publishes no sampler number; BASELINE.md says the yardstick is
"a plain eager PyTorch-ROCm implementation of the same math, measured on the
same MI355X".  This is that implementation: the reference's loop
(ViT.py:220-237) verbatim in behaviour — per step a host-built timestep tensor,
the module-by-module nn.Linear / softmax / LayerNorm forward
(``forward_reference``), clamp, eps-hat and the DDIM update as separate
elementwise ops — in fp32 (the reference samples without autocast) or under
bf16 autocast.
"""
from __future__ import annotations

import math
import time

import torch


@torch.no_grad()
def eager_ddim_sample(model, device, k: int, N: int, generator=None, autocast_bf16: bool = False,
                      device_noise: bool = False, noise=None):
    """``noise``: start from this x_T (on ``device``) instead of drawing one."""
    T = model.total_steps
    C, (H, W) = model.in_chans, model.img_size
    if noise is not None:
        x = noise.to(device).float()
    elif device_noise:  # same noise policy as the fused sampler under comparison
        x = torch.randn((N, C, H, W), device=device, generator=generator)
    else:
        x = torch.normal(0.0, 1.0, (N, C, H, W), generator=generator).to(device)
    x0 = x
    for t in range(T - 1, 0, -k):
        tt = torch.tensor([t] * N, device=device)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast_bf16):
            x0 = model.forward_reference(x, tt)
        x0 = torch.clamp(x0.float(), -1.0, 1.0)
        a_tk = 1 - math.sqrt((t + 1 - k) / T)
        a_t = 1 - math.sqrt((t + 1) / T) + 1e-5
        eps = (x - math.sqrt(a_t) * x0) / math.sqrt(1 - a_t)
        x = math.sqrt(a_tk) * (x / math.sqrt(a_t) + (math.sqrt((1 - a_tk) / a_tk) - math.sqrt((1 - a_t) / a_t)) * eps)
    return (x0.cpu() + 1) / 2


def time_eager_sampler(model, device, k: int, N: int, reps: int = 2, autocast_bf16: bool = False,
                       device_noise: bool = False) -> float:
    """Seconds per N-image batch (after one warm-up batch)."""
    was = model.training
    model.eval()
    try:
        g = torch.Generator(device=device if device_noise else "cpu").manual_seed(0)
        eager_ddim_sample(model, device, k, N, g, autocast_bf16, device_noise)
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        for _ in range(reps):
            eager_ddim_sample(model, device, k, N, g, autocast_bf16, device_noise)
        torch.cuda.synchronize(device)
        return (time.perf_counter() - t0) / reps
    finally:
        model.train(was)


@torch.no_grad()
def eager_img2img(model, device, draft, starts, k: int, eps):
    """The reference's draft->drawing loop (ViT_draft2drawing.py:394-409): one
    t_start at a time at batch 1, fp32 eager forward, host-side coefficients and
    a host-built timestep tensor per step.  ``draft`` [1,C,H,W] / ``eps``
    [len(starts),C,H,W] on ``device``; returns the final clamped x0-hat per start
    (device, [-1, 1])."""
    T = model.total_steps
    outs = []
    for i, t_start in enumerate(starts):
        a = 1 - math.sqrt(t_start / T)
        x = math.sqrt(1 - a) * eps[i:i + 1] + math.sqrt(a) * draft
        x0 = x
        for t in range(t_start, 0, -k):
            x0 = torch.clamp(model.forward_reference(x, torch.tensor([t], device=device)), -1.0, 1.0)
            a_tk = 1 - math.sqrt((t + 1 - k) / T)
            a_t = 1 - math.sqrt((t + 1) / T) + 1e-5
            e = (x - math.sqrt(a_t) * x0) / math.sqrt(1 - a_t)
            x = math.sqrt(a_tk) * (x / math.sqrt(a_t) + (math.sqrt((1 - a_tk) / a_tk) - math.sqrt((1 - a_t) / a_t)) * e)
        outs.append(x0)
    return torch.cat(outs)


def time_img2img(model, device, starts, k: int, reps: int = 5, eager: bool = False) -> float:
    """Seconds per draft->drawing call over ``starts`` (fused: one replayed hipGraph
    of the batched loop, noise drawn on the host and the result copied back as
    :func:`ddim_cold_amd.diffusion.samplers.img2img` does; ``eager``: the
    reference's sequential batch-1 loop, one call)."""
    from ..diffusion.samplers import img2img
    was = model.training
    model.eval()
    try:
        g = torch.Generator().manual_seed(0)
        C, (H, W) = model.in_chans, model.img_size
        draft = torch.rand(1, C, H, W, generator=g, device="cpu").to(device) * 2 - 1
        if eager:
            eps = torch.randn(len(starts), C, H, W, generator=g).to(device)
            eager_img2img(model, device, draft, starts[:1], k, eps)  # warm-up
            torch.cuda.synchronize(device)
            t0 = time.perf_counter()
            out = eager_img2img(model, device, draft, starts, k, eps)
            out.cpu()
            return time.perf_counter() - t0
        img2img(model, draft, starts, k=k, device=device, generator=g)  # warm-up + capture
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        for _ in range(reps):
            img2img(model, draft, starts, k=k, device=device, generator=g)
        torch.cuda.synchronize(device)
        return (time.perf_counter() - t0) / reps
    finally:
        model.train(was)
