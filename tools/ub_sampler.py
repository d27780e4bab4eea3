"""DDIM sampler (k=20, N=64, ViT-tiny) ms per batch, A/B of a samplers.py module switch,
interleaved in one process: python tools/ub_sampler.py PATCH_CHAIN [reps] [rounds]"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd import build_model
from ddim_cold_amd.diffusion import samplers as smp

flag = sys.argv[1] if len(sys.argv) > 1 else "PATCH_CHAIN"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 3
torch.manual_seed(1234)
model = build_model("vit_tiny").cuda().eval()
noise = torch.randn(64, 3, 64, 64, generator=torch.Generator().manual_seed(0))
res = {True: [], False: []}
for r in range(rounds):
    for on in (True, False):
        setattr(smp, flag, on)
        model.__dict__.pop("_sampler_graphs", None)
        s = smp.DDIMSampler(model, "cuda", k=20)
        s.sample(64, noise=noise)  # capture
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            s.sample(64, noise=noise)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / reps * 1e3
        res[on].append(ms)
        print(f"round {r} {flag}={on}: {ms:.3f} ms/batch", flush=True)
for on in (True, False):
    v = sorted(res[on])
    print(f"{flag}={on}: median {v[len(v) // 2]:.3f} ms/batch  ({', '.join(f'{x:.2f}' for x in res[on])})")
