"""Input-gradient GEMM dX = dY W (W stored [out][in], the "transposed B" LDS-DMA path,
ds_read_b64_tr_b16 fragments) vs the same product with W^T stored k-contiguous (the
forward's non-transposed path), graph-timed, at the training shapes.

    python tools/ub_dgrad_layout.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ddim_cold_amd import ops  # noqa: E402
from tools.ubench import t  # noqa: E402

dev = "cuda"
torch.manual_seed(0)
for M in (20032, 2080):
    for out, inn, f32 in ((1152, 384, True), (1152, 384, False), (384, 384, False)):
        dy = (torch.randn(M, out, device=dev)).to(torch.bfloat16)
        w = (torch.randn(out, inn, device=dev) * 0.05).to(torch.bfloat16)
        wt = w.t().contiguous()
        a = t(lambda: ops.linear_dgrad(dy, w, f32))
        b = t(lambda: ops.linear_fwd(dy, wt, None, f32))
        d = (ops.linear_dgrad(dy, w, f32).float() - ops.linear_fwd(dy, wt, None, f32).float()).abs().max().item()
        fl = 2 * M * out * inn
        print(f"M={M:6d} K={out:5d} N={inn}: W (transposed-B path) {a:6.2f} us  W^T (forward path) {b:6.2f} us"
              f"  ({fl / a / 1e6:4.0f} vs {fl / b / 1e6:4.0f} TF, max|d| {d:.1e}, {'f32' if f32 else 'bf16'} out)", flush=True)
# input gradient through GELU (fc2): dU = (dY W) * gelu'(u), dropout p = 0.1
r = torch.tensor([1, 2], dtype=torch.int64, device=dev)
for M in (20032, 2080):
    dy = torch.randn(M, 384, device=dev).to(torch.bfloat16)
    w = (torch.randn(384, 384, device=dev) * 0.05).to(torch.bfloat16)
    u = torch.randn(M, 384, device=dev).to(torch.bfloat16)
    wt = w.t().contiguous()
    a = t(lambda: ops.linear_dgrad_gelu(dy, w, u, r, 11, 0.1))
    b = t(lambda: ops.linear_dgrad_gelu(dy, w, u, r, 11, 0.1, wt=wt))
    print(f"dgelu M={M:6d} K=384 N=384: W {a:6.2f} us  W^T {b:6.2f} us", flush=True)
