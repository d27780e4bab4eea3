"""Where a DDIM k=20 N=64 sample() call spends its time: the whole call vs the bare
graph replay, and the host-side pieces (state lookup, noise draw, result copy)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd import build_model
from ddim_cold_amd.diffusion.samplers import DDIMSampler

model = build_model("vit_tiny").cuda().eval()
s = DDIMSampler(model, "cuda", k=20)
g = torch.Generator(device="cuda").manual_seed(0)
s.sample(64, generator=g, device_noise=True)
torch.cuda.synchronize()


def t(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


st = s._state(64, False)
res = {
    "sample() call": t(lambda: s.sample(64, generator=g, device_noise=True)),
    "graph replay only": t(lambda: st["loop"].graph.replay()),
    "_state() lookup (host)": t(lambda: s._state(64, False)),
    "noise draw": t(lambda: st["x"].normal_(0.0, 1.0, generator=g)),
    "result to host": t(lambda: st["x0"].add(1.0).div_(2.0).cpu()),
}
for k, v in res.items():
    print(f"{v:8.3f} ms  {k}")
