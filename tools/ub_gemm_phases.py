"""Per-phase GEMM timing (main loop vs epilogue) via DDIM_COLD_GEMM_DEBUG."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd import ops
from tools.ubench import t
dev = "cuda"
M, D, B, N, H = 2080, 384, 32, 65, 12
def bf(*s, sc=1.0): return (torch.randn(*s, device=dev) * sc).to(torch.bfloat16)
a, w, b = bf(M, D), bf(D, D, sc=0.05), torch.randn(D, device=dev)
w3, b3 = bf(3 * D, D, sc=0.05), torch.randn(3 * D, device=dev)
x = torch.randn(M, D, device=dev)
r = torch.tensor([1, 2], dtype=torch.int64, device=dev)
dqkv = bf(M, 3 * D)
res = {
 "resid": t(lambda: ops.linear_residual_fwd(a, w, b, x, N, r, 3, 0.0, 4, 0.0)),
 "qkv": t(lambda: ops.qkv_fwd(a, w3, b3, B, N, H)),
 "plain nt bf16 2080x1152": t(lambda: ops.linear_fwd(a, w3, b3, False)),
 "plain nt f32 2080x1152": t(lambda: ops.linear_fwd(a, w3, b3, True)),
 "plain nt bf16 2080x384": t(lambda: ops.linear_fwd(a, w, b, False)),
 "gelu": t(lambda: ops.linear_gelu_fwd(a, w, b, r, 5, 0.0)),
 "dgrad f32": t(lambda: ops.linear_dgrad(a, w, True)),
 "dgrad qkv": t(lambda: ops.linear_dgrad(dqkv, w3, True)),
}
print(os.environ.get("DDIM_COLD_GEMM_DEBUG", "0"), {k: round(v, 2) for k, v in res.items()})
