import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd import ops
from tools.ubench import t
dev = "cuda"
M, D, N = 2080, 384, 65
def bf(*s, sc=1.0): return (torch.randn(*s, device=dev) * sc).to(torch.bfloat16)
a, w, b = bf(M, D), bf(D, D, sc=0.05), torch.randn(D, device=dev)
x = torch.randn(M, D, device=dev); g0, b0 = torch.randn(D, device=dev), torch.randn(D, device=dev)
r = torch.tensor([1, 2], dtype=torch.int64, device=dev)
print(os.environ.get("DDIM_COLD_LN_GEMM_DEBUG", "0"), "p=0.1", round(t(lambda: ops.linear_residual_ln_fwd(a, w, b, x, g0, b0, 1e-5, N, r, 3, 0.1, 4, 0.1)), 2),
      "p=0", round(t(lambda: ops.linear_residual_ln_fwd(a, w, b, x, g0, b0, 1e-5, N, r, 3, 0., 4, 0.)), 2))
