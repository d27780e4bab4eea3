"""Is the transposed-operand (token-major) weight-gradient GEMM slower than the
same product with K-contiguous operands?  dW[1152,384] = dY^T X over 2080 tokens:
  (a) grouped wgrad kernel on dY [2080,1152], X [2080,384]   (both operands transposed)
  (b) forward NT GEMM on dY^T [1152,2080], X^T [384,2080]    (both K-contiguous)"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd import ops
from tools.ubench import t
dev = "cuda"
M, D = 2080, 384
res = {}
for n in (1152, 384):
    dy = torch.randn(M, n, device=dev).to(torch.bfloat16)
    x = torch.randn(M, D, device=dev).to(torch.bfloat16)
    dw = torch.zeros(n, D, device=dev)
    dyT, xT = dy.t().contiguous(), x.t().contiguous()
    res[f"wgrad-T {n}x{D}"] = round(t(lambda: ops.linear_wgrad_group([(dy, x, dw, None)])), 2)
    res[f"nt-gemm {n}x{D}"] = round(t(lambda: ops.linear_fwd(dyT, xT, None, True)), 2)
    torch.testing.assert_close(ops.linear_fwd(dyT, xT, None, True), dy.float().t() @ x.float(), rtol=1e-2, atol=1e-1)
print(os.environ.get("DDIM_COLD_WGRAD_GROUP_SPLITS", "auto"), res)
