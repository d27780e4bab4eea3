"""Phase timeline of the short attention backward (ViT-tiny training shape): wave 0 of
every workgroup stamps s_memrealtime (100 MHz) at start / after the loads+LDS images /
after the query phase / at the end.  Prints medians over workgroups (ns).
Needs a stamps build (compiled out by default):
    DDIM_COLD_HIPFLAGS=-DDDIM_COLD_ATTN_STAMPS=1 python -m ddim_cold_amd.build
"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd import ops
from ddim_cold_amd.ops._ext import load
load()
C = torch.ops.ddim_cold
dev = "cuda"
B, H, N, hd = 32, 12, 65, 32
torch.manual_seed(0)
qkv = (torch.randn(3, B, H, N, hd, device=dev)).to(torch.bfloat16)
do = torch.randn(B, N, H * hd, device=dev).to(torch.bfloat16)
r = torch.tensor([1, 2], dtype=torch.int64, device=dev)
for p in (0.1, 0.0):
    keep = ops.attn_keep_buffer(qkv, p)
    o, lse = ops.attn_fwd(qkv, hd ** -0.5, r, 5, p, keep_out=keep)
    st = torch.zeros(B * H, 4, dtype=torch.int64, device=dev)
    for it in range(3):  # last run counts (warm)
        C.attn_stamps(st)
        ops.attn_bwd(do, qkv, o, lse, hd ** -0.5, r, 5, p, keep=keep)
        torch.cuda.synchronize()
        C.attn_stamps(None)
    s = st.double() * 10.0  # ns
    t0 = s[:, 0].min()
    med = lambda x: float(x.median())
    print(f"p={p}: start spread {med(s[:, 0] - t0):.0f} ns (max {float((s[:, 0] - t0).max()):.0f}); "
          f"loads+images {med(s[:, 1] - s[:, 0]):.0f}; query phase {med(s[:, 2] - s[:, 1]):.0f}; "
          f"key phase {med(s[:, 3] - s[:, 2]):.0f}; total per WG {med(s[:, 3] - s[:, 0]):.0f}; "
          f"kernel span {float(s[:, 3].max() - t0):.0f} ns", flush=True)
# start-offset distribution of the last run (p = 0): percentiles, per XCD (blockIdx % 8)
off = (s[:, 0] - t0)
q = torch.quantile(off, torch.tensor([0.1, 0.25, 0.5, 0.75, 0.9, 0.95, 0.99], dtype=torch.float64, device=off.device))
print("start offset percentiles (ns) 10/25/50/75/90/95/99:", [round(float(v)) for v in q])
for x in range(8):
    o = off[x::8]
    print(f"xcd {x}: median {float(o.median()):.0f} max {float(o.max()):.0f} late(>3us) {int((o > 3000).sum())}")
late = (off > 3000).nonzero().flatten().tolist()
print("late block ids:", late[:40], "count", len(late))
