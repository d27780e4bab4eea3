"""Per-k-tile cost of the grouped weight-gradient kernel vs the token count
(working set): dW[1152,384] = dY^T X over T tokens, 64x64 tiles, no split."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd import ops
from tools.ubench import t
dev = "cuda"
for T in (256, 512, 1024, 2080, 4160):
    dy = torch.randn(T, 1152, device=dev).to(torch.bfloat16)
    x = torch.randn(T, 384, device=dev).to(torch.bfloat16)
    dw = torch.zeros(1152, 384, device=dev)
    us = t(lambda: ops.linear_wgrad_group([(dy, x, dw, None)]))
    print(f"T={T} kt={(T + 63) // 64} us={us:.2f} per-kt={(us - 4) / ((T + 63) // 64):.3f}")
