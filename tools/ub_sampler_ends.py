"""Sampler head (EPI 5, DDIM update + bf16 patch rows) and patch-embed (EPI 6,
patches_in) GEMMs at the ViT-tiny N=64 sampler shape, graph-timed.  Run once per
setting of DDIM_COLD_GEMM_DEBUG (1: main loop only, 2: epilogue only) / _TILE.
Prints one JSON line {label: us}."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd import ops
from tools.ubench import t

dev = "cuda"
torch.manual_seed(0)
rng = torch.tensor([1, 2], dtype=torch.int64, device=dev)
B, D, P, C, HW = 64, 384, 8, 3, 64
NP = (HW // P) ** 2
N = NP + 1
M = B * N
F = C * P * P
res = {}
xb = (torch.randn(M, D, device=dev)).to(torch.bfloat16)
st = torch.rand(M, D // 32, 2, device=dev) + 1.0
hw = (torch.randn(F, D, device=dev) * 0.05).to(torch.bfloat16)
hb = torch.randn(F, device=dev)
hc = torch.randn(F, device=dev)
x = torch.randn(B, C, HW, HW, device=dev)
x0 = torch.empty_like(x)
coef = torch.tensor([0.5, 0.8, 0.6, 0.7], device=dev)
pout = torch.empty(B * NP, F, dtype=torch.bfloat16, device=dev)
res["head_step mode1 +patches"] = t(lambda: ops.head_step_(xb, hw, hb, x, x0, coef, P, 1, fold=(st, hc, 1e-5),
                                                           patches_out=pout))
xr = ops.image_to_rows(x, P).contiguous()
x0r = torch.empty_like(xr)
res["head_rows mode1 +patches"] = t(lambda: ops.head_step_rows_(xb, hw, hb, xr, x0r, coef, B, 1, fold=(st, hc, 1e-5),
                                                                patches_out=pout))
res["head_rows mode1"] = t(lambda: ops.head_step_rows_(xb, hw, hb, xr, x0r, coef, B, 1, fold=(st, hc, 1e-5)))
res["head_step mode1"] = t(lambda: ops.head_step_(xb, hw, hb, x, x0, coef, P, 1, fold=(st, hc, 1e-5)))
pe_w = (torch.randn(D, F, device=dev) * 0.05).to(torch.bfloat16)
pe_b, cls = torch.randn(D, device=dev), torch.randn(D, device=dev)
pos, temb = torch.randn(N, D, device=dev), torch.randn(2000, D, device=dev)
tt = torch.randint(0, 2000, (B,), device=dev)
lst = torch.empty(M, D // 32, 2, device=dev)
xbo = torch.empty(M, D, dtype=torch.bfloat16, device=dev)
res["embed patches_in"] = t(lambda: ops.patch_embed_fwd(x, tt, pe_w, pe_b, cls, pos, temb, rng, 1, 0.0, P,
                                                        ln_st=lst, xb_out=xbo, patches_in=pout))
res["embed patchify"] = t(lambda: ops.patch_embed_fwd(x, tt, pe_w, pe_b, cls, pos, temb, rng, 1, 0.0, P,
                                                      ln_st=lst, xb_out=xbo))
res["empty"] = t(lambda: rng.add_(0))
tag = " ".join(f"{k}={os.environ[k]}" for k in ("DDIM_COLD_GEMM_DEBUG", "DDIM_COLD_GEMM_TILE") if k in os.environ)
print(json.dumps({"env": tag or "default", **{k: round(v, 2) for k, v in res.items()}}))
