"""DDIM sampler (k=20, N=64) per GEMM tile configuration (ops.gemm_tile, captured per
config; -1 = the automatic choice) on a model config: which tile family the sampler-sized
GEMMs want (usage: python tools/ub_sampler_tiles.py [model] [tiles, e.g. -1,1,4])."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ddim_cold_amd import ops  # noqa: E402
from ddim_cold_amd.diffusion.samplers import DDIMSampler  # noqa: E402
from ddim_cold_amd.models import build_model  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "oxford_flower"
tiles = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [-1, 1, 4]
dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = build_model(name).to(dev).eval()
for tile in tiles:
    model.__dict__.pop("_sampler_graphs", None)  # captured loops are cached per model
    with ops.gemm_tile(tile):
        s = DDIMSampler(model, dev, k=20)
        g = torch.Generator(device=dev).manual_seed(0)
        s.sample(64, generator=g, device_noise=True)  # capture under this tile config
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            s.sample(64, generator=g, device_noise=True)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 10
    print(f"{name} tile {tile}: {dt * 1e3:.2f} ms per batch, {64 / dt:.1f} img/s", flush=True)
    del s
