"""PMC / timing target: the long-sequence attention kernels (flash forward, dq / dkv
backward) on the high-resolution shapes, 10 eager calls each.

    N = 626  : vit_small_200 (200x200, p=8, 6 heads x 64), per-GPU batch 32
    N = 2501 : 200x200 at p=4, 4 heads x 64, batch 8

argv[1] = "time": graph-timed fwd/bwd us + TFLOP/s per shape (no profiler needed).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd import ops

dev = "cuda"
r = torch.tensor([1, 2], dtype=torch.int64, device=dev)
SHAPES = [(32, 6, 626, 64), (8, 4, 2501, 64)]
mode = sys.argv[1] if len(sys.argv) > 1 else "pmc"
for (B, H, N, hd) in SHAPES:
    torch.manual_seed(0)
    qkv = (torch.randn(3, B, H, N, hd, device=dev) * 0.5).to(torch.bfloat16)
    do = torch.randn(B, N, H * hd, device=dev).to(torch.bfloat16)
    for p in (0.0, 0.1):
        o, lse = ops.attn_fwd(qkv, hd ** -0.5, r, 5, p)
        if mode == "time":
            from tools.ubench import t
            f = t(lambda: ops.attn_fwd(qkv, hd ** -0.5, r, 5, p), reps=10)
            b = t(lambda: ops.attn_bwd(do, qkv, o, lse, hd ** -0.5, r, 5, p), reps=10)
            fl = 4 * B * H * N * N * hd  # QK^T + PV, 2 flop per MAC
            print(f"B{B} H{H} N{N} hd{hd} p{p}: fwd {f:.1f} us {fl / f / 1e6:.1f} TFLOP/s | "
                  f"bwd {b:.1f} us {2.5 * fl / b / 1e6:.1f} TFLOP/s", flush=True)
        else:
            for _ in range(10):
                ops.attn_fwd(qkv, hd ** -0.5, r, 5, p)
                ops.attn_bwd(do, qkv, o, lse, hd ** -0.5, r, 5, p)
torch.cuda.synchronize()
print("ok")
