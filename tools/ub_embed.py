"""Patch-embedding GEMM (EPI_EMBED) cost breakdown at the sampler shape (B=64) and the
training shape (B=32): graph-timed (tools/ubench.py's timer)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd import ops, build_model
from ddim_cold_amd.models.program import model_tensors
from ubench import t as timeit

torch.manual_seed(0)
model = build_model("vit_tiny").cuda().eval()
P = model_tensors(model)
r = torch.zeros(2, dtype=torch.int64, device="cuda")
for B in (64, 32):
    img = torch.randn(B, 3, 64, 64, device="cuda")
    tt = torch.randint(0, 2000, (B,), device="cuda")
    N, D = 65, 384
    st = torch.empty(B * N, D // 32, 2, device="cuda")
    xb = torch.empty(B * N, D, dtype=torch.bfloat16, device="cuda")
    _, pin = ops.patch_embed_fwd(img, tt, P.pe_w, P.pe_b, P.cls, P.pos, P.temb, r, 0, 0.0, 8)
    res = {}
    res["patchify+gemm, fold producer"] = timeit(lambda: ops.patch_embed_fwd(img, tt, P.pe_w, P.pe_b, P.cls, P.pos, P.temb, r, 0, 0.0, 8, ln_st=st, xb_out=xb))
    res["gemm+cls rows (patches_in), fold producer"] = timeit(lambda: ops.patch_embed_fwd(img, tt, P.pe_w, P.pe_b, P.cls, P.pos, P.temb, r, 0, 0.0, 8, ln_st=st, xb_out=xb, patches_in=pin))
    res["patchify+gemm, no fold"] = timeit(lambda: ops.patch_embed_fwd(img, tt, P.pe_w, P.pe_b, P.cls, P.pos, P.temb, r, 0, 0.0, 8))
    res["plain bf16 GEMM same shape"] = timeit(lambda: ops.linear_fwd(pin, P.pe_w, None, False))
    for k, v in res.items():
        print(f"B={B}: {v:7.2f} us  {k}")
