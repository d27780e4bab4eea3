"""The reference CLI's default sampling call (ViT.py: sample_n=256, acc_k=1 -> 2,000 denoiser
steps at N=256) on the graph-captured sampler: capture+first run time, replay time, memory."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd import build_model
from ddim_cold_amd.diffusion.samplers import DDIMSampler

model = build_model(sys.argv[1] if len(sys.argv) > 1 else "oxford_flower").cuda().eval()
s = DDIMSampler(model, "cuda", k=1)
g = torch.Generator(device="cuda").manual_seed(0)
torch.cuda.synchronize()
t0 = time.perf_counter()
out = s.sample(256, generator=g, device_noise=True)
torch.cuda.synchronize()
t1 = time.perf_counter()
out2 = s.sample(256, generator=g, device_noise=True)
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"steps {len(s.ts)}  first call (eager warm-up + capture) {t1 - t0:.2f} s  replay {t2 - t1:.2f} s "
      f"({256 / (t2 - t1):.1f} img/s)  max mem {torch.cuda.max_memory_allocated() / 2**30:.2f} GiB  "
      f"finite {bool(torch.isfinite(out2).all())} range [{out2.min():.3f}, {out2.max():.3f}]")
