"""LayerNorm backward in isolation (graph-timed, tools/ubench.t) at the training
shapes: bf16 dy (dgrad hand-off) and bf16 x (the folded forward's copy), fp32
residual gradient in / out, gy (dropout p + drop-path), y_out (LayerNorm output for
the folded GEMM's weight gradient), slot workspace.  Bytes moved and the rate.

    python tools/ub_ln_bwd.py [M,N ...]   (default 20032,626 2080,65)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ddim_cold_amd import ops  # noqa: E402
from ddim_cold_amd.ops import reference as ref  # noqa: E402
from tools.ubench import t  # noqa: E402

dev = "cuda"
shapes = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]] or [(20032, 626), (2080, 65)]
D = 384
for M, N in shapes:
    torch.manual_seed(0)
    x = torch.randn(M, D, device=dev)
    g, b = torch.randn(D, device=dev), torch.randn(D, device=dev)
    _, mu, rs = ref.layernorm_fwd(x, g, b)
    xb = x.to(torch.bfloat16)
    dy = torch.randn(M, D, device=dev).to(torch.bfloat16)
    gres = torch.randn(M, D, device=dev)
    r = torch.tensor([1, 2], dtype=torch.int64, device=dev)
    ws = torch.zeros(ops.ln_ws_rows(M), 2 * D, device=dev)
    y = torch.empty(M, D, dtype=torch.bfloat16, device=dev)
    z = torch.zeros(D, device=dev)
    fn = lambda: ops.layernorm_bwd(dy, xb, mu, rs, g, gres, z, z, N, r, 7, 0.1, 8, 0.1, True, ws, beta=b, y_out=y)
    us = t(fn)
    byts = M * D * (2 + 2 + 4) + M * D * (4 + 2 + 2)  # in: dy, x, g_res; out: g_out, gy, y_out
    print(f"ln_bwd M={M} D={D}: {us:7.2f} us  {byts / 1e6:6.1f} MB  {byts / us / 1e6:5.2f} TB/s", flush=True)
