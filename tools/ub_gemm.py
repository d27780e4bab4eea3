"""GEMM shape sweep: time(M, N, K) for our dgrad-path GEMM (fp32 out) and hipBLASLt."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd import ops
from tools.ubench import t
dev = "cuda"
def bf(*s, sc=1.0): return (torch.randn(*s, device=dev) * sc).to(torch.bfloat16)
for (M, N, K) in [(2080, 1152, 64), (2080, 1152, 384), (2080, 1152, 1152), (2080, 384, 64), (2080, 384, 384),
                  (2080, 384, 1152), (8320, 384, 384), (8320, 1152, 384), (4160, 384, 384)]:
    a = bf(M, K); w = bf(K, N, sc=0.05)   # dgrad: dx[M,N] = a[M,K] @ w[K,N]
    wt = w.t().contiguous()
    ours_bt = t(lambda: ops.linear_dgrad(a, w, True))
    xres = torch.zeros(M, N, device=dev)
    ours_nt = t(lambda: ops.linear_residual_fwd(a, wt, torch.zeros(N, device=dev), xres, 65 if M % 65 == 0 else 1, torch.zeros(2, dtype=torch.int64, device=dev), 0, 0.0, 0, 0.0))
    blas = t(lambda: torch.matmul(a, w))
    fl = 2 * M * N * K
    print(f"M={M:5d} N={N:5d} K={K:5d}  ours(BT,f32)={ours_bt:7.2f}us ({fl/ours_bt/1e6:6.1f} TF)  ours(NT,resid)={ours_nt:7.2f}us  hipblaslt={blas:7.2f}us ({fl/blas/1e6:6.1f} TF)", flush=True)
