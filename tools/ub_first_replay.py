"""Cost of the FIRST replays of a freshly captured K-step training graph vs the later
ones (the driver times 20 steps = 5 replays right after a 5-step warm-up that never
replays the K-step graph), optionally after a GEMM burn that ramps the GPU clocks.
Results: profiles/first_replay_r6.txt.

    python tools/ub_first_replay.py [vit_tiny] [burn_ms]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from ddim_cold_amd import build_model
from ddim_cold_amd.data.synthetic import ColdBatcher, synthetic_pool
from ddim_cold_amd.train import engine as E

name = sys.argv[1] if len(sys.argv) > 1 else "vit_tiny"
burn_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
if burn_ms > 0:  # keep the GPU busy before the warm-up (clock ramp hypothesis)
    a = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < burn_ms:
        for _ in range(10):
            a = (a @ a).clamp_(-1, 1)
        torch.cuda.synchronize()
    del a
torch.manual_seed(0)
m = build_model(name).cuda().train()
eng = E.TrainEngine(m, E.EngineConfig(lr=1e-3, t_max=51200, seed=42, temb_rows=7, graph_steps=4))
eng.set_batch_fn(ColdBatcher(synthetic_pool(1024, tuple(m.img_size), seed=7, device="cuda"), 32, eng.rng))
eng.train_steps(5)  # the bench warm-up: 3 eager steps, capture, single-step replays
torch.cuda.synchronize()
ts = []
for _ in range(8):
    t0 = time.perf_counter()
    eng.train_steps(4)
    torch.cuda.synchronize()
    ts.append((time.perf_counter() - t0) * 1e3 / 4)
print(f"{name} burn={burn_ms:g}ms: ms/step per 4-step replay: " + " ".join(f"{t:.4f}" for t in ts), flush=True)
