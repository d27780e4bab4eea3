"""PMC target: the training step's hot kernels on the ViT-tiny shapes, 20 calls each (eager)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd import ops

dev = "cuda"
torch.manual_seed(0)
M, D, B, N, H = 2080, 384, 32, 65, 12
r = torch.tensor([1, 2], dtype=torch.int64, device=dev)


def bf(*s, sc=1.0):
    return (torch.randn(*s, device=dev) * sc).to(torch.bfloat16)


a, w, b = bf(M, D), bf(D, D, sc=0.05), torch.randn(D, device=dev)
w3, b3 = bf(3 * D, D, sc=0.05), torch.randn(3 * D, device=dev)
x = torch.randn(M, D, device=dev)
g, be = torch.randn(D, device=dev), torch.randn(D, device=dev)
dqkv = bf(M, 3 * D)
def job(nout, k, m=M):
    return (bf(m, nout, sc=0.1), bf(m, k, sc=0.1), torch.zeros(nout, k, device=dev), torch.zeros(nout, device=dev))


# the step's deferred weight-gradient launch: 7 blocks (qkv, proj, fc1, fc2) + head + patch embedding
wjobs = [job(3 * D, D) if i % 4 == 0 else job(D, D) for i in range(28)] + [job(192, D), job(D, 192, 2048)]
qkv = bf(3, B, H, N, 32)
do = bf(B, N, D)
u = bf(M, D)
_, mu, rs = ops.layernorm_fwd(x, g, be)
ws = torch.zeros(ops.ln_ws_rows(M), 2 * D, device=dev)
dyb = bf(M, D)
keep = ops.attn_keep_buffer(qkv, 0.1)
n = 7_300_000
p_, g_, m_, v_ = [torch.randn(n, device=dev) for _ in range(4)]
pb = torch.empty(n, device=dev, dtype=torch.bfloat16)
sq = torch.zeros(1024, device=dev)
st = torch.zeros(2, dtype=torch.int64, device=dev)
hy = torch.tensor([1e-4, 0.9, 0.999, 1e-8, 0.05, 1.0, 1000.0, 0.0], device=dev)
for _ in range(20):
    ops.linear_residual_fwd(a, w, b, x, N, r, 3, 0.1, 4, 0.1)
    ops.qkv_fwd(a, w3, b3, B, N, H)
    ops.linear_gelu_fwd(a, w, b, r, 5, 0.1)
    ops.linear_dgrad(dqkv, w3, True)
    ops.linear_dgrad(a, w, False)
    ops.linear_dgrad_gelu(a, w, u, r, 5, 0.1)
    ops.linear_wgrad_multi(wjobs, store=True)
    o, lse = ops.attn_fwd(qkv, 32 ** -0.5, r, 5, 0.1, keep_out=keep)
    ops.attn_bwd(do, qkv, o, lse, 32 ** -0.5, r, 5, 0.1, keep=keep)
    ops.layernorm_bwd(dyb, x, mu, rs, g, x, g.clone(), be.clone(), N, r, 3, 0.1, 4, 0.1, True, ws)
    ops.sqnorm(g_, sq, 1.0)
    ops.adamw_step(p_, g_, m_, v_, pb, sq, st, hy, 1.0)
torch.cuda.synchronize()
print("ok")
