"""Grouped weight-gradient GEMM of one ViT-tiny block (qkv 1152x384, proj/fc1/fc2
384x384, K = 2080 tokens), graph-timed.  Env (read once per process):
DDIM_COLD_WGRAD_GROUP_SPLITS, DDIM_COLD_GEMM_DEBUG (1 skip epilogue, 2 skip main loop)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd import ops
from tools.ubench import t
dev = "cuda"
M, D = 2080, 384
def bf(*s): return torch.randn(*s, device=dev).to(torch.bfloat16)
jobs = []
for n in (3 * D, D, D, D):
    jobs.append((bf(M, n), bf(M, D), torch.zeros(n, D, device=dev), torch.zeros(n, device=dev)))
us = t(lambda: ops.linear_wgrad_group(jobs))
print("splits", os.environ.get("DDIM_COLD_WGRAD_GROUP_SPLITS", "auto"), "debug",
      os.environ.get("DDIM_COLD_GEMM_DEBUG", "0"), round(us, 2))
