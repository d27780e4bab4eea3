"""Per-workgroup phase timeline of the LDS-DMA GEMM (csrc/gemm.hip gemm_dma_body
stamps, ops gemm_stamps): start -> first operand stage ready -> main loop done ->
epilogue done, per workgroup, plus which CU ran it.  Shapes: the vit_small_200 step
(M = 20,032 token rows, D = 384) and the ViT-tiny step (M = 2,080).
usage: python tools/ub_gemm_stamps.py [M (default 20032)] [tile configs, e.g. -1,4,5,3,1 (ops.gemm_tile)]
Needs a stamps build of the extension (the stamp code costs the production step ~1.5 %):
  DDIM_COLD_HIPFLAGS=-DDDIM_COLD_GEMM_STAMPS python -m ddim_cold_amd.build --force"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ddim_cold_amd import ops  # noqa: E402

dev = "cuda"
M = int(sys.argv[1]) if len(sys.argv) > 1 else 20032
D = 384
B = 32
N, H = M // B, 6 if M > 8192 else 12
torch.manual_seed(0)
T = torch.ops.ddim_cold


def bf(*s, sc=1.0):
    return (torch.randn(*s, device=dev) * sc).to(torch.bfloat16)


r = torch.tensor([1, 2], dtype=torch.int64, device=dev)
a = bf(M, D)
w, b = bf(D, D, sc=0.05), torch.randn(D, device=dev)
w3, b3 = bf(3 * D, D, sc=0.05), torch.randn(3 * D, device=dev)
x = torch.randn(M, D, device=dev)
st = torch.empty(M, D // 32, 2, device=dev)
xb = torch.empty(M, D, dtype=torch.bfloat16, device=dev)
st_in = torch.rand(M, D // 32, 2, device=dev) + 1.0
c3, c1 = torch.randn(3 * D, device=dev), torch.randn(D, device=dev)
mean, rstd = torch.empty(M, device=dev), torch.empty(M, device=dev)
dy3 = bf(M, 3 * D)
cases = [
    ("qkv fwd (LN fold, head-major)", lambda: ops.qkv_fwd(a, w3, b3, B, N, H, fold=(st_in, c3, 1e-5, mean, rstd))),
    ("fc1 GELU (LN fold, dropout)", lambda: ops.linear_gelu_fwd(a, w, b, r, 3, 0.1, fold=(st_in, c1, 1e-5, mean, rstd))),
    ("proj residual (dropout, drop-path, stats)", lambda: ops.linear_residual_fwd(a, w, b, x, N, r, 4, 0.1, 5, 0.1,
                                                                                  st_out=st, xb_out=xb)),
    ("dgrad bf16 K=384", lambda: ops.linear_dgrad(a, w, False)),
    ("dgrad fp32 K=1152", lambda: ops.linear_dgrad(dy3, w3, True)),
    ("plain bf16", lambda: ops.linear_fwd(a, w, b)),
]
TILES = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [-1]
buf = torch.zeros(6 << 17, dtype=torch.int32, device=dev)
for (name0, fn), tile in [(c, tl) for c in cases for tl in TILES]:
    name = name0 + ("" if tile < 0 else f" [tile cfg {tile}]")
    with ops.gemm_tile(tile):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        buf.zero_()
        T.gemm_stamps(buf)
        fn()
        torch.cuda.synchronize()
        T.gemm_stamps(None)
    s = buf.view(-1, 6)
    s = s[s[:, 3] != 0].to(torch.int64).cpu()
    if s.numel() == 0:
        print(name, ": no stamps (not an LDS-DMA launch, or the extension was built without "
              "-DDDIM_COLD_GEMM_STAMPS)")
        continue
    t0 = s[:, 0].min()
    st0, st1, st2, st3 = ((s[:, i] - t0).float() * 0.01 for i in range(4))  # 100 MHz -> us
    hw, xcc = s[:, 4], s[:, 5]
    cu = (xcc & 0xF) * 1000 + ((hw >> 13) & 7) * 100 + ((hw >> 12) & 1) * 50 + ((hw >> 8) & 0xF)
    n = s.shape[0]
    q = lambda v: f"{v.median().item():5.2f} [{v.quantile(0.1).item():5.2f}, {v.quantile(0.9).item():5.2f}]"
    ncu = cu.unique().numel()
    per = torch.bincount(torch.unique(cu, return_inverse=True)[1])
    print(f"{name}: {n} workgroups on {ncu} CUs (max {per.max().item()} per CU), span {st3.max().item():.2f} us")
    print(f"   start offset {q(st0)} | wait for first stage {q(st1 - st0)} | main loop {q(st2 - st1)} | "
          f"epilogue {q(st3 - st2)} | total {q(st3 - st0)}  (median [p10, p90] us)")
    # consecutive workgroups on one CU: gap between one's end and the next's start
    gaps = []
    for c in cu.unique().tolist():
        idx = (cu == c).nonzero().flatten()
        order = st0[idx].argsort()
        ss, ee = st0[idx][order], st3[idx][order]
        for i in range(1, len(ss)):
            gaps.append((ss[i] - ee[i - 1]).item())
    if gaps:
        g = torch.tensor(gaps)
        print(f"   next workgroup on the same CU starts {g.median().item():.2f} us after the previous ends "
              f"(p10 {g.quantile(0.1).item():.2f}, p90 {g.quantile(0.9).item():.2f}; negative = overlapping)")
