"""Profiling target: graph-replayed DDIM k=20 N=64 sampling (ViT-tiny), 3 timed calls."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd import build_model
from ddim_cold_amd.diffusion.samplers import DDIMSampler

model = build_model("vit_tiny").cuda().eval()
s = DDIMSampler(model, "cuda", k=20)
g = torch.Generator(device="cuda").manual_seed(0)
for _ in range(4):
    s.sample(64, generator=g, device_noise=True)
torch.cuda.synchronize()
print("ok")
