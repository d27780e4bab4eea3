"""Profiling target: eager DDIM k=20 N=64 sampling of a named model (argv[1])."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd import build_model
from ddim_cold_amd.diffusion.samplers import DDIMSampler

model = build_model(sys.argv[1] if len(sys.argv) > 1 else "oxford_flower").cuda().eval()
s = DDIMSampler(model, "cuda", k=20, use_graph=False)
for _ in range(2):
    s.sample(64)
torch.cuda.synchronize()
print("ok")
