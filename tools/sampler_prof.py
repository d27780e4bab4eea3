"""Profiling target: 3 eager (non-graph) DDIM k=20 N=64 sampling batches of ViT-tiny."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd import build_model
from ddim_cold_amd.diffusion.samplers import DDIMSampler

model = build_model("vit_tiny").cuda().eval()
s = DDIMSampler(model, "cuda", k=20, use_graph=False)
for _ in range(3):
    s.sample(64)
torch.cuda.synchronize()
print("ok")
