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
                      device_noise: bool = False):
    T = model.total_steps
    C, (H, W) = model.in_chans, model.img_size
    if device_noise:  # same noise policy as the fused sampler under comparison
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
