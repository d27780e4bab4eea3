"""How much of the training step is dropout / drop-path: graph-timed engine step
of ViT-tiny (B=32) with the reference's rates vs all rates 0 (diagnostic only)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd.models import build_model
from ddim_cold_amd.train.engine import EngineConfig, TrainEngine
from ddim_cold_amd.data.synthetic import ColdBatcher, synthetic_pool


def run(**kw):
    torch.manual_seed(0)
    m = build_model("vit_tiny", **kw).cuda().train()
    eng = TrainEngine(m, EngineConfig(lr=3e-4, t_max=1000, temb_rows=7))
    eng.set_batch_fn(ColdBatcher(synthetic_pool(1024, device="cuda"), 32, eng.rng))
    for _ in range(20):
        eng.train_step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        eng.train_step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / 200 * 1e3


for rep in range(2):
    a = run()
    b = run(drop_rate=0.0, attn_drop_rate=0.0, drop_path_rate=0.0)
    c = run(drop_rate=0.1, attn_drop_rate=0.0, drop_path_rate=0.1)
    print(f"ms/step  reference rates {a:.4f}   no dropout {b:.4f}   no attention dropout {c:.4f}", flush=True)
