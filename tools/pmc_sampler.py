"""PMC target: the DDIM sampler's per-step kernels on the ViT-tiny N=64 shapes (eval:
no dropout), 20 eager calls each -- M = 64 x 65 = 4160 token rows.  Collected by
tools/gpu_pmc_sampler.sh; summarised by tools/pmc_waves.py."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd import ops

dev = "cuda"
torch.manual_seed(0)
B, N, D, H = 64, 65, 384, 12
M = B * N
r = torch.tensor([1, 2], dtype=torch.int64, device=dev)


def bf(*s, sc=1.0):
    return (torch.randn(*s, device=dev) * sc).to(torch.bfloat16)


a, w, b = bf(M, D), bf(D, D, sc=0.05), torch.randn(D, device=dev)
w3, b3 = bf(3 * D, D, sc=0.05), torch.randn(3 * D, device=dev)
x = torch.randn(M, D, device=dev)
qkv = bf(3, B, H, N, 32)
for _ in range(20):
    ops.qkv_fwd(a, w3, b3, B, N, H)
    ops.attn_fwd(qkv, 32 ** -0.5, r, 5, 0.0)
    ops.linear_residual_fwd(a, w, b, x, N, r, 3, 0.0, 4, 0.0)
    ops.linear_gelu_fwd(a, w, b, r, 5, 0.0)
torch.cuda.synchronize()
print("ok")
