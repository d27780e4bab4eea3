"""Large-M GEMMs of the vit_small_200 training step (M = B*N = 32*626 = 20,032 token rows,
D = 384) for every tile config (ops.gemm_tile; -1 = automatic choice) vs hipBLASLt
(torch.matmul, bf16 out) on the same shapes; graph-timed (tools/ubench.t).
usage: python tools/ub_gemm_large.py [M] [tiles, e.g. -1,1,4,5] [D (default 384)]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ddim_cold_amd import ops  # noqa: E402
from tools.ubench import t  # noqa: E402

dev = "cuda"
M = int(sys.argv[1]) if len(sys.argv) > 1 else 20032
TILES = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [-1, 1, 3, 4, 5]
D = int(sys.argv[3]) if len(sys.argv) > 3 else 384
B, H = 32, D // 64
N = M // B
torch.manual_seed(0)


def bf(*s, sc=1.0):
    return (torch.randn(*s, device=dev) * sc).to(torch.bfloat16)


r = torch.tensor([1, 2], dtype=torch.int64, device=dev)
a = bf(M, D)
w, b = bf(D, D, sc=0.05), torch.randn(D, device=dev)
w3, b3 = bf(3 * D, D, sc=0.05), torch.randn(3 * D, device=dev)
x = torch.randn(M, D, device=dev)
w4, b4 = bf(4 * D, D, sc=0.05), torch.randn(4 * D, device=dev)
w4t, h4 = bf(D, 4 * D, sc=0.05), bf(M, 4 * D)
dq = bf(M, 3 * D)
st = torch.empty(M, D // 32, 2, device=dev)
xb = torch.empty(M, D, dtype=torch.bfloat16, device=dev)
fl1 = 2 * M * D * D
fl3 = 2 * M * D * 3 * D
cases = [
    ("qkv fwd (head-major scatter)", fl3, lambda: ops.qkv_fwd(a, w3, b3, B, N, H), lambda: torch.matmul(a, w3.t())),
    ("plain bf16 out N=3D", fl3, lambda: ops.linear_fwd(a, w3, b3), None),
    ("gelu fwd p=0 (3D x D)", fl3, lambda: ops.linear_gelu_fwd(a, w3, b3, r, 5, 0.0), None),
    ("resid fwd p=.1 dp=.1 +stats", fl1,
     lambda: ops.linear_residual_fwd(a, w, b, x, N, r, 3, 0.1, 4, 0.1, st_out=st, xb_out=xb),
     lambda: torch.matmul(a, w.t())),
    ("gelu fwd p=0.1 (D x D)", fl1, lambda: ops.linear_gelu_fwd(a, w, b, r, 5, 0.1), None),
    ("gelu fwd p=0 (4D x D)", 4 * fl1, lambda: ops.linear_gelu_fwd(a, w4, b4, r, 5, 0.0), None),
    ("resid fwd K=4D", 4 * fl1, lambda: ops.linear_residual_fwd(h4, w4t, b, x, N, r, 3, 0.0, 4, 0.0),
     lambda: torch.matmul(h4, w4t.t())),
    ("dgrad K=384 bf16 out", fl1, lambda: ops.linear_dgrad(a, w, False), lambda: torch.matmul(a, w)),
    ("dgrad K=384 f32 out", fl1, lambda: ops.linear_dgrad(a, w, True), None),
    ("dgrad-gelu p=0.1", fl1, lambda: ops.linear_dgrad_gelu(a, w, xb, r, 11, 0.1), None),
    ("dgrad qkv K=1152 f32 out", fl3, lambda: ops.linear_dgrad(dq, w3, True), lambda: torch.matmul(dq, w3)),
]
for name, fl, fn, blas in cases:
    s = f"{name:30s}"
    ref_out = None
    for tile in TILES:
        with ops.gemm_tile(tile):
            us = t(fn)
            out = fn()
        o = out[0] if isinstance(out, tuple) else out
        if ref_out is None:
            ref_out = o.float().clone()
        dif = (o.float() - ref_out).abs().max().item()
        s += f" | t{tile}: {us:6.1f} us {fl / us / 1e6:5.0f} TF" + (f" d={dif:.1e}" if dif > 0 else "")
    if blas is not None:
        bu = t(blas)
        s += f" | hipBLASLt {bu:6.1f} us {fl / bu / 1e6:5.0f} TF"
    print(s, flush=True)
