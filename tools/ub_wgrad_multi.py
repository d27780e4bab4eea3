"""Graph-timed micro-benchmark of the whole-backward weight-gradient launch
(ops.linear_wgrad_multi) on the ViT-tiny step's problem set and subsets."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd import ops
from tools.ubench import t

dev = "cuda"
M, D = 2080, 384
def bf(*s): return (torch.randn(*s, device=dev) * 0.1).to(torch.bfloat16)
def job(nout, k, m=M): return (bf(m, nout), bf(m, k), torch.zeros(nout, k, device=dev), torch.zeros(nout, device=dev))
blocks = [[job(3 * D, D), job(D, D), job(D, D), job(D, D)] for _ in range(7)]
head, pe = job(192, D), job(D, 192, 2048)
full = [j for b in blocks for j in b] + [head, pe]
sets = {"full (1548 tiles)": full, "no head (1530)": full[:-2] + [pe], "blocks only (1512)": full[:-2],
        "6 blocks (1296)": [j for b in blocks[:6] for j in b], "1 block (216)": blocks[0],
        "qkv x7 (756)": [b[0] for b in blocks]}
for name, js in sets.items():
    print(f"{t(lambda: ops.linear_wgrad_multi(js), reps=20):8.2f} us  {name}")
