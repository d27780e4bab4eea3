"""Phase timeline of the LayerNorm backward (ViT-tiny training shape, bf16 dy, replica
workspace, re-emitted LayerNorm output): thread 0 of every workgroup stamps
s_memrealtime (100 MHz) at start / first row's loads landed / row stores issued / LDS
column partials staged / replica atomics issued.  Medians over workgroups (ns).

Needs a stamps build (compiled out by default):
    DDIM_COLD_HIPFLAGS=-DDDIM_COLD_LN_STAMPS=1 python -m ddim_cold_amd.build
"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd import ops
from ddim_cold_amd.ops._ext import load
load()
C = torch.ops.ddim_cold
dev = "cuda"
M, D, N = 2080, 384, 65
torch.manual_seed(0)
x = torch.randn(M, D, device=dev)
g, be = torch.randn(D, device=dev), torch.randn(D, device=dev)
_, mu, rs = ops.layernorm_fwd(x, g, be)
dyb = (torch.randn(M, D, device=dev)).to(torch.bfloat16)
ws = torch.zeros(ops.LN_REPLICAS, 2 * D, device=dev)
yo = torch.empty(M, D, dtype=torch.bfloat16, device=dev)
r = torch.tensor([1, 2], dtype=torch.int64, device=dev)
grid = (M + 7) // 8
st = torch.zeros(grid, 5, dtype=torch.int64, device=dev)
for it in range(3):
    C.ln_stamps(st)
    ops.layernorm_bwd(dyb, x, mu, rs, g, x, g.clone(), be.clone(), N, r, 3, 0.1, 4, 0.1, True, ws, beta=be, y_out=yo)
    torch.cuda.synchronize()
    C.ln_stamps(None)
s = st.double() * 10.0
t0 = s[:, 0].min()
med = lambda v: float(v.median())
print(f"start spread median {med(s[:, 0] - t0):.0f} max {float((s[:, 0] - t0).max()):.0f} ns; loads {med(s[:, 1] - s[:, 0]):.0f}; "
      f"rows {med(s[:, 2] - s[:, 1]):.0f}; LDS stage {med(s[:, 3] - s[:, 2]):.0f}; atomics {med(s[:, 4] - s[:, 3]):.0f}; "
      f"per WG {med(s[:, 4] - s[:, 0]):.0f}; span {float(s[:, 4].max() - t0):.0f} ns", flush=True)
