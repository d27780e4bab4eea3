"""Forward GEMM phases on the sampler (M=4160) and training (M=2080) ViT-tiny shapes,
graph-timed: run once per setting of the GEMM switches (read once per process):

    DDIM_COLD_GEMM_DEBUG=1   main loop only (no epilogue stores)
    DDIM_COLD_GEMM_DEBUG=2   epilogue only (no main loop)
    DDIM_COLD_GEMM_TILE=0..3 force 32x64 / 64x64 / 128x64 / 128x128

Prints one JSON line {label: us}."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd import ops
from tools.ubench import t

dev = "cuda"
torch.manual_seed(0)
r = torch.tensor([1, 2], dtype=torch.int64, device=dev)
D, H, N = 384, 12, 65
res = {}


def bf(*s, sc=1.0):
    return (torch.randn(*s, device=dev) * sc).to(torch.bfloat16)


for B in (32, 64):
    M = B * N
    a, w, b = bf(M, D), bf(D, D, sc=0.05), torch.randn(D, device=dev)
    w3, b3 = bf(3 * D, D, sc=0.05), torch.randn(3 * D, device=dev)
    x = torch.randn(M, D, device=dev)
    res[f"qkv M={M}"] = t(lambda: ops.qkv_fwd(a, w3, b3, B, N, H))
    # LayerNorm-folded consumers / producer, as in the model
    st = torch.rand(M, D // 32, 2, device=dev) + 1.0
    c3, c1 = torch.randn(3 * D, device=dev), torch.randn(D, device=dev)
    mo, ro = torch.empty(M, device=dev), torch.empty(M, device=dev)
    so, xo = torch.empty(M, D // 32, 2, device=dev), torch.empty(M, D, dtype=torch.bfloat16, device=dev)
    res[f"qkv fold M={M}"] = t(lambda: ops.qkv_fwd(a, w3, b3, B, N, H, fold=(st, c3, 1e-5, mo, ro)))
    res[f"gelu fold M={M}"] = t(lambda: ops.linear_gelu_fwd(a, w, b, r, 5, 0.0, fold=(st, c1, 1e-5, mo, ro)))
    res[f"resid prod M={M}"] = t(lambda: ops.linear_residual_fwd(a, w, b, x, N, r, 3, 0.0, 4, 0.0, st_out=so,
                                                                 xb_out=xo))
    res[f"resid M={M}"] = t(lambda: ops.linear_residual_fwd(a, w, b, x, N, r, 3, 0.0, 4, 0.0))
    res[f"gelu M={M}"] = t(lambda: ops.linear_gelu_fwd(a, w, b, r, 5, 0.0))
res["empty"] = t(lambda: r.add_(0))
tag = " ".join(f"{k}={os.environ[k]}" for k in ("DDIM_COLD_GEMM_DEBUG", "DDIM_COLD_GEMM_TILE") if k in os.environ)
print(json.dumps({"env": tag or "default", **{k: round(v, 2) for k, v in res.items()}}))
