"""Per-op microbenchmark: HIP kernels vs hipBLASLt (torch.matmul) on the ViT-tiny shapes."""
import sys, os, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd import ops
dev = "cuda"
if __name__ != "__main__":
    pass
GRAPH = os.environ.get("UB_EAGER", "0") != "1"


def t(fn, reps=50, warm=5):
    """Device time per call: `reps` calls captured in one graph, replayed 10x."""
    for _ in range(warm): fn()
    torch.cuda.synchronize()
    if not GRAPH:
        s, e = torch.cuda.Event(True), torch.cuda.Event(True)
        s.record()
        for _ in range(reps): fn()
        e.record(); torch.cuda.synchronize()
        return s.elapsed_time(e) / reps * 1e3
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps): fn()
    g.replay(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(10): g.replay()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / (10 * reps) * 1e3


def main():
    torch.manual_seed(0)
    M, D, B, N, H = 2080, 384, 32, 65, 12
    r = torch.tensor([1, 2], dtype=torch.int64, device=dev)

    def bf(*s, sc=1.0): return (torch.randn(*s, device=dev) * sc).to(torch.bfloat16)
    a, w, b = bf(M, D), bf(D, D, sc=0.05), torch.randn(D, device=dev)
    w3, b3 = bf(3 * D, D, sc=0.05), torch.randn(3 * D, device=dev)
    x = torch.randn(M, D, device=dev)
    res = {}
    res["hipblaslt mm 2080x384x384"] = t(lambda: torch.matmul(a, w.t()))
    res["hipblaslt mm 2080x1152x384"] = t(lambda: torch.matmul(a, w3.t()))
    res["hipblaslt mm 384x384x2080 (wgrad)"] = t(lambda: torch.matmul(a.t(), a))
    res["resid p=0.1"] = t(lambda: ops.linear_residual_fwd(a, w, b, x, N, r, 3, 0.1, 4, 0.1))
    res["resid p=0"] = t(lambda: ops.linear_residual_fwd(a, w, b, x, N, r, 3, 0.0, 4, 0.0))
    g0, b0 = torch.randn(D, device=dev), torch.randn(D, device=dev)
    a2, x2 = bf(2 * M, D), torch.randn(2 * M, D, device=dev)
    res["resid M=4160 p=0"] = t(lambda: ops.linear_residual_fwd(a2, w, b, x2, N, r, 3, 0.0, 4, 0.0))
    res["ln fwd M=4160"] = t(lambda: ops.layernorm_fwd(x2, g0, b0))
    res["qkv"] = t(lambda: ops.qkv_fwd(a, w3, b3, B, N, H))
    res["plain bf16 out 2080x1152 (qkv shape, EPI_BF16 via dgrad-free path)"] = t(lambda: ops.linear_dgrad(a, w3.t().contiguous(), False))
    k0 = torch.zeros(M, 0, device=dev, dtype=torch.bfloat16)
    res["gelu"] = t(lambda: ops.linear_gelu_fwd(a, w, b, r, 5, 0.1))
    res["dgrad f32"] = t(lambda: ops.linear_dgrad(a, w, True))
    res["dgrad bf16"] = t(lambda: ops.linear_dgrad(a, w, False))
    dqkv = bf(M, 3 * D)
    res["dgrad qkv (K=1152)"] = t(lambda: ops.linear_dgrad(dqkv, w3, True))
    dw, db = torch.zeros(D, D, device=dev), torch.zeros(D, device=dev)
    res["wgrad 384x384"] = t(lambda: ops.linear_wgrad(a, a, dw, db))
    dw3, db3 = torch.zeros(3 * D, D, device=dev), torch.zeros(3 * D, device=dev)
    res["wgrad 1152x384"] = t(lambda: ops.linear_wgrad(dqkv, a, dw3, db3))
    h_ = bf(M, D)
    blk = [(a, h_, dw, db), (a, h_, dw.clone(), db.clone()), (a, h_, dw.clone(), db.clone()), (dqkv, a, dw3, db3)]
    res["wgrad multi (block: 3x384^2 + 1152x384)"] = t(lambda: ops.linear_wgrad_multi(blk))
    g, bb = torch.randn(D, device=dev), torch.randn(D, device=dev)
    res["ln fwd"] = t(lambda: ops.layernorm_fwd(x, g, bb))
    _, mu, rs = ops.layernorm_fwd(x, g, bb)
    dg, dbb = torch.zeros(D, device=dev), torch.zeros(D, device=dev)
    res["ln bwd"] = t(lambda: ops.layernorm_bwd(x, x, mu, rs, g, x, dg, dbb, N, r, 3, 0.1, 4, 0.1, True))
    qkv = bf(3, B, H, N, 32)
    res["attn fwd"] = t(lambda: ops.attn_fwd(qkv, 32 ** -0.5, r, 5, 0.1))
    o, lse = ops.attn_fwd(qkv, 32 ** -0.5, r, 5, 0.1)
    do = bf(B, N, D)
    res["attn bwd"] = t(lambda: ops.attn_bwd(do, qkv, o, lse, 32 ** -0.5, r, 5, 0.1))
    img = torch.randn(B, 3, 64, 64, device=dev)
    res["smooth_l1"] = t(lambda: ops.smooth_l1_fwd_bwd(img, img * 0.5, N, 8))
    gg = torch.randn(B, N, D, device=dev); tt = torch.randint(0, 2000, (B,), device=dev)
    dcls, dpos, dtemb = torch.zeros(D, device=dev), torch.zeros(N, D, device=dev), torch.zeros(2000, D, device=dev)
    res["embed bwd"] = t(lambda: ops.embed_bwd(gg, tt, r, 1, 0.1, dcls, dpos, dtemb))
    n = 7_300_000
    p_, g_, m_, v_ = [torch.randn(n, device=dev) for _ in range(4)]
    pb = torch.empty(n, device=dev, dtype=torch.bfloat16); sq = torch.zeros(1024, device=dev)
    st = torch.zeros(2, dtype=torch.int64, device=dev)
    hy = torch.tensor([1e-4, 0.9, 0.999, 1e-8, 0.05, 1.0, 1000.0, 0.0], device=dev)
    res["sqnorm 7.3M"] = t(lambda: ops.sqnorm(g_, sq, 1.0))
    res["adamw 7.3M"] = t(lambda: ops.adamw_step(p_, g_, m_, v_, pb, sq, st, hy, 1.0))
    res["empty kernel (torch fill 1 elem)"] = t(lambda: sq.zero_())
    for k, v in res.items():
        print(f"{v:8.2f} us  {k}")
    print(json.dumps({k: round(v, 2) for k, v in res.items()}))


if __name__ == "__main__":
    main()
