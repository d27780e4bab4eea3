"""Attention fwd/bwd timings on the model shapes (graph-timed): ViT-tiny train / sampler
(N=65), OxfordFlower (N=257), vit_small_200 (N=626), 200x200 at p=4 (N=2501).
DDIM_COLD_LIB=<other .so> times another build."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd import ops
from tools.ubench import t
dev = "cuda"
r = torch.tensor([1, 2], dtype=torch.int64, device=dev)
res = {}
SHAPES = [(32, 12, 65, 32), (64, 12, 65, 32), (32, 4, 257, 64), (64, 4, 257, 64), (32, 6, 626, 64), (8, 4, 2501, 64)]
for (B, H, N, hd) in SHAPES:
    qkv = (torch.randn(3, B, H, N, hd, device=dev) * 0.5).to(torch.bfloat16)
    do = (torch.randn(B, N, H * hd, device=dev)).to(torch.bfloat16)
    for p in (0.0, 0.1):
        for stored in ((False, True) if p > 0 else (False,)):
            keep = ops.attn_keep_buffer(qkv, p) if stored else None
            if stored and keep is None:
                continue
            o, lse = ops.attn_fwd(qkv, hd ** -0.5, r, 5, p, keep_out=keep)
            f = t(lambda: ops.attn_fwd(qkv, hd ** -0.5, r, 5, p, keep_out=keep), reps=20)
            b = t(lambda: ops.attn_bwd(do, qkv, o, lse, hd ** -0.5, r, 5, p, keep=keep), reps=20)
            fl = 4 * B * H * N * N * hd
            row = {"fwd_us": round(f, 1), "bwd_us": round(b, 1),
                   "fwd_TFLOPs": round(fl / f / 1e6, 1), "bwd_TFLOPs": round(2.5 * fl / b / 1e6, 1)}
            res[f"B{B} H{H} N{N} hd{hd} p{p}" + (" stored-masks" if stored else "")] = row
for k, v in res.items():
    print(k, v)
