"""Fused MLP block vs the two-GEMM launches, graph-timed, on the model shapes.

    python tools/ub_mlp.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from ddim_cold_amd import ops
from tools.ubench import t

dev = "cuda"
r = torch.tensor([1, 2], dtype=torch.int64, device=dev)
for (M, D, H, N, pd, save, name) in [(2080, 384, 384, 65, 0.1, True, "ViT-tiny train B=32"),
                                     (4160, 384, 384, 65, 0.0, False, "ViT-tiny sampler N=64"),
                                     (16448, 256, 256, 257, 0.0, False, "oxford sampler N=64"),
                                     (40064, 384, 384, 626, 0.0, False, "vit_small_200 sampler N=64"),
                                     (20032, 384, 384, 626, 0.1, True, "vit_small_200 train B=32")]:
    x1 = torch.randn(M, D, device=dev)
    xb = x1.to(torch.bfloat16)
    st = torch.randn(M, D // 32, 2, device=dev).abs() * 30 + 10
    w1 = (torch.randn(H, D, device=dev) * 0.05).to(torch.bfloat16)
    c1, b1 = torch.randn(H, device=dev), torch.randn(H, device=dev)
    w2 = (torch.randn(D, H, device=dev) * 0.05).to(torch.bfloat16)
    b2 = torch.randn(D, device=dev)
    so, xo = torch.empty(M, D // 32, 2, device=dev), torch.empty(M, D, dtype=torch.bfloat16, device=dev)
    m2, r2 = torch.empty(M, device=dev), torch.empty(M, device=dev)
    res = {}
    for bm in (0, 16, 32, 64):
        res[f"fused bm{bm or 'auto'}"] = t(lambda: ops.mlp_fused_fwd(xb, x1, st, w1, c1, b1, w2, b2, 1e-5, N, r, 1, 2, pd,
                                                                     3, pd, save, so, xo, m2, r2, bm=bm), reps=20)

    def two():
        u, h = ops.linear_gelu_fwd(xb, w1, b1, r, 1, pd, fold=(st, c1, 1e-5, m2, r2))
        return ops.linear_residual_fwd(h, w2, b2, x1, N, r, 2, pd, 3, pd, st_out=so, xb_out=xo)
    res["two GEMMs"] = t(two, reps=20)
    fl = 4 * M * D * H
    print(f"{name} (M={M}, D={D}, H={H}): " + "  ".join(f"{k} {v:.1f} us ({fl / v / 1e6:.0f} TF/s)"
                                                       for k, v in res.items()), flush=True)
