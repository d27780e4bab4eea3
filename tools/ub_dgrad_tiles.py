"""Tile configurations (ops.gemm_tile; -1 = automatic) for the input-gradient GEMMs on
transposed weight shadows at vit_small_200's M = 20,032: plain (QKV K = 1,152 fp32 out,
K = 384 bf16 out) and through GELU (fc2).  Graph-timed."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ddim_cold_amd import ops  # noqa: E402
from tools.ubench import t  # noqa: E402

dev = "cuda"
torch.manual_seed(0)
M = 20032
r = torch.tensor([1, 2], dtype=torch.int64, device=dev)
cases = []
for out, f32 in ((1152, True), (384, False)):
    dy = torch.randn(M, out, device=dev).to(torch.bfloat16)
    wt = (torch.randn(384, out, device=dev) * 0.05).to(torch.bfloat16)
    cases.append((f"dgrad K={out}", lambda dy=dy, wt=wt, f32=f32: ops.linear_fwd(dy, wt, None, f32)))
dy = torch.randn(M, 384, device=dev).to(torch.bfloat16)
u = torch.randn(M, 384, device=dev).to(torch.bfloat16)
wt = (torch.randn(384, 384, device=dev) * 0.05).to(torch.bfloat16)
cases.append(("dgelu", lambda: ops.linear_dgrad_gelu(dy, None, u, r, 11, 0.1, wt=wt)))
for name, fn in cases:
    s = f"{name:14s}"
    ref_out = None
    for tile in (-1, 0, 1, 2, 3, 4, 5, 6):
        with ops.gemm_tile(tile):
            us = t(fn)
            o = fn().float()
        if ref_out is None:
            ref_out = o
        d = (o - ref_out).abs().max().item()
        s += f" | t{tile}: {us:6.2f}" + (f" d={d:.0e}" if d > 1e-2 else "")
    print(s, flush=True)
