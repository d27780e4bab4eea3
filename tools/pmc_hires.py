"""PMC target: the vit_small_200 training step's hot kernels (M = 32 x 626 = 20,032 token
rows, D = 384, 6 heads x 64, MLP ratio 1), 5 calls each (eager): the QKV projection
(256x192 tiles), the residual GEMM, the input gradients on transposed weight shadows (QKV,
through GELU), the long-sequence attention forward (dropout keep words stored) and its dQ /
dK-dV backward kernels, the LayerNorm backward and the 8-wave weight-gradient launch (one
block's four problems x 6: 324 tiles, split tail)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from ddim_cold_amd import ops  # noqa: E402

dev = "cuda"
torch.manual_seed(0)
B, N, H, D = 32, 626, 6, 384
M, hd = B * N, D // H
r = torch.tensor([1, 2], dtype=torch.int64, device=dev)


def bf(*s, sc=1.0):
    return (torch.randn(*s, device=dev) * sc).to(torch.bfloat16)


a, w, b = bf(M, D), bf(D, D, sc=0.05), torch.randn(D, device=dev)
w3, b3 = bf(3 * D, D, sc=0.05), torch.randn(3 * D, device=dev)
x = torch.randn(M, D, device=dev)
g, be = torch.randn(D, device=dev), torch.randn(D, device=dev)
dqkv = bf(M, 3 * D)
u = bf(M, D)
qkv = bf(3, B, H, N, hd)
do = bf(B, N, D)
_, mu, rs = ops.layernorm_fwd(x, g, be)
ws = torch.zeros(ops.ln_ws_rows(M), 2 * D, device=dev)
w3t = w3.t().contiguous()
wt = w.t().contiguous()
dyb = bf(M, D)
keep = ops.attn_keep_buffer(qkv, 0.1)


def job(nout, k):
    return (bf(M, nout, sc=0.1), bf(M, k, sc=0.1), torch.zeros(nout, k, device=dev), torch.zeros(nout, device=dev))


wjobs = [job(3 * D, D), job(D, D), job(D, D), job(D, D)] * 6  # six blocks' weight gradients
for _ in range(5):
    ops.qkv_fwd(a, w3, b3, B, N, H)
    ops.linear_residual_fwd(a, w, b, x, N, r, 3, 0.1, 4, 0.1)
    ops.linear_fwd(dqkv, w3t, None, True)  # QKV input gradient on the transposed shadow
    ops.linear_dgrad_gelu(dyb, w, u, r, 11, 0.1, wt=wt)
    o, lse = ops.attn_fwd(qkv, hd ** -0.5, r, 5, 0.1, keep_out=keep)
    ops.attn_bwd(do, qkv, o, lse, hd ** -0.5, r, 5, 0.1, keep=keep)
    ops.layernorm_bwd(dyb, x, mu, rs, g, x, g.clone(), be.clone(), N, r, 3, 0.1, 4, 0.1, True, ws)
    ops.linear_wgrad_multi(wjobs, store=True)
torch.cuda.synchronize()
print("ok")
