"""DDIM k=20 N=64 sampler throughput vs number of concurrent chains (streams)."""
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd import build_model
from ddim_cold_amd.diffusion.samplers import DDIMSampler

model = build_model("vit_tiny").cuda().eval()
N = int(os.environ.get("UB_N", "64"))
for streams in [1, 2, 3, 4, 8]:
    s = DDIMSampler(model, "cuda", k=20, streams=streams)
    s.sample(N)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        s.sample(N)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 5
    print(f"streams {streams}: {dt * 1e3:7.2f} ms/batch  {N / dt:8.1f} img/s", flush=True)
