"""LayerNorm backward timing on the ViT-tiny shape (one config per process:
DDIM_COLD_LN_BWD_CFG is read once by the extension)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd import ops
from tools.ubench import t
dev = "cuda"
M, D, N = 2080, 384, 65
x, dy, gr = (torch.randn(M, D, device=dev) for _ in range(3))
mean, rstd = x.mean(1), torch.rsqrt(x.var(1, unbiased=False) + 1e-5)
g, dg, db = (torch.randn(D, device=dev) for _ in range(3))
ws = torch.zeros(ops.LN_REPLICAS, 2 * D, device=dev)
r = torch.tensor([1, 2], dtype=torch.int64, device=dev)
res = {}
for p in (0.0, 0.1):
    res[p] = round(t(lambda: ops.layernorm_bwd(dy, x, mean, rstd, g, gr, dg, db, N, r, 3, p, 4, p, True, ws=ws)), 2)
print("cfg", os.environ.get("DDIM_COLD_LN_BWD_CFG", "0"), res)
y = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
if hasattr(ops, "layernorm_fwd"):
    b0 = torch.randn(D, device=dev)
    print("fwd waves", os.environ.get("DDIM_COLD_LN_FWD_WAVES", "4"),
          round(t(lambda: ops.layernorm_fwd(x, g, b0, 1e-5)), 2))
