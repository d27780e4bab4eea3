"""Profiling target: DDIM k=20 N=64 sampling batches (graph-replayed after one capture) of a
model config (default ViT-tiny): python tools/sampler_prof.py [model] [batches]."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from ddim_cold_amd import build_model  # noqa: E402
from ddim_cold_amd.diffusion.samplers import DDIMSampler  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "vit_tiny"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
model = build_model(name).cuda().eval()
s = DDIMSampler(model, "cuda", k=20)
for _ in range(reps):
    s.sample(64)
torch.cuda.synchronize()
print("ok")
