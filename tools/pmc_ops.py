"""PMC target: a few GEMM/LN/attention ops, 20 calls each (eager)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd import ops
dev = "cuda"
torch.manual_seed(0)
M, D, B, N, H = 2080, 384, 32, 65, 12
r = torch.tensor([1, 2], dtype=torch.int64, device=dev)
def bf(*s, sc=1.0): return (torch.randn(*s, device=dev) * sc).to(torch.bfloat16)
a, w, b = bf(M, D), bf(D, D, sc=0.05), torch.randn(D, device=dev)
w3, b3 = bf(3 * D, D, sc=0.05), torch.randn(3 * D, device=dev)
x = torch.randn(M, D, device=dev)
dw, db = torch.zeros(D, D, device=dev), torch.zeros(D, device=dev)
for _ in range(20):
    ops.linear_residual_fwd(a, w, b, x, N, r, 3, 0.1, 4, 0.1)
    ops.qkv_fwd(a, w3, b3, B, N, H)
    ops.linear_dgrad(a, w, True)
    ops.linear_wgrad(a, a, dw, db)
torch.cuda.synchronize()
print("ok")
