"""Dropout cost per kernel: the ViT-tiny training shapes with p = 0.1 vs p = 0
(graph-timed, tools/ubench.py's timer).  The difference bounds what a cheaper
mask hash could save."""
import sys, os, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd import ops
from ubench import t

dev = "cuda"


def main():
    torch.manual_seed(0)
    M, D, B, N, H = 2080, 384, 32, 65, 12
    r = torch.tensor([1, 2], dtype=torch.int64, device=dev)

    def bf(*s, sc=1.0): return (torch.randn(*s, device=dev) * sc).to(torch.bfloat16)
    a, w, b = bf(M, D), bf(D, D, sc=0.05), torch.randn(D, device=dev)
    x = torch.randn(M, D, device=dev)
    qkv = bf(3, B, H, N, 32)
    do = bf(B, N, D)
    g, bb = torch.randn(D, device=dev), torch.randn(D, device=dev)
    _, mu, rs = ops.layernorm_fwd(x, g, bb)
    dg, dbb = torch.zeros(D, device=dev), torch.zeros(D, device=dev)
    res = {}
    for p in (0.1, 0.0):
        res[f"resid p={p}"] = t(lambda: ops.linear_residual_fwd(a, w, b, x, N, r, 3, p, 4, p))
        res[f"gelu p={p}"] = t(lambda: ops.linear_gelu_fwd(a, w, b, r, 5, p))
        res[f"attn fwd p={p}"] = t(lambda: ops.attn_fwd(qkv, 32 ** -0.5, r, 5, p))
        o, lse = ops.attn_fwd(qkv, 32 ** -0.5, r, 5, p)
        res[f"attn bwd p={p}"] = t(lambda: ops.attn_bwd(do, qkv, o, lse, 32 ** -0.5, r, 5, p))
        kb = ops.attn_keep_buffer(qkv, p)
        if kb is not None:
            res[f"attn fwd p={p} +store keep"] = t(lambda: ops.attn_fwd(qkv, 32 ** -0.5, r, 5, p, keep_out=kb))
            res[f"attn bwd p={p} stored keep"] = t(lambda: ops.attn_bwd(do, qkv, o, lse, 32 ** -0.5, r, 5, p, keep=kb))
        res[f"ln bwd p={p}"] = t(lambda: ops.layernorm_bwd(x, x, mu, rs, g, x, dg, dbb, N, r, 3, p, 4, p, True))
    for k, v in res.items():
        print(f"{v:8.2f} us  {k}")
    print(json.dumps({k: round(v, 2) for k, v in res.items()}))


if __name__ == "__main__":
    main()
