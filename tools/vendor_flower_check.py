"""oxford_flower vendor comparator inside a bench-like process (after our engine trained) vs alone."""
import sys, torch
sys.path.insert(0, ".")
from ddim_cold_amd.bench.vendor_baseline import time_vendor_train
from ddim_cold_amd.data.synthetic import synthetic_pool, ColdBatcher
from ddim_cold_amd.models import build_model
from ddim_cold_amd.train.engine import EngineConfig, TrainEngine
dev = torch.device("cuda", 0)
mode = sys.argv[1]
pool = synthetic_pool(1024, (64, 64), seed=7, device=dev)
if mode == "after_engine":
    torch.manual_seed(0)
    m = build_model("oxford_flower").to(dev).train()
    eng = TrainEngine(m, EngineConfig(lr=3.125e-4, t_max=51200, use_graph=True, graph_steps=4))
    eng.set_batch_fn(ColdBatcher(pool, 32, eng.rng))
    eng.train_steps(220)
    torch.cuda.synchronize()
    print("engine loss", float(eng.loss_ema), flush=True)
from ddim_cold_amd.bench.vendor_baseline import VendorTrainStep  # noqa: E402
for patch in ("conv", "gemm"):
    for sync in (False, True):
        torch.manual_seed(1234)
        vm = build_model("oxford_flower").to(dev).train()
        v = VendorTrainStep(vm, pool, 32, 3.125e-4, 51200, patch=patch)
        for i in range(220):
            v.steps(1)
            if sync:
                torch.cuda.synchronize()
        print(mode, "patch", patch, "sync every replay" if sync else "back to back", "loss", float(v.loss),
              "non-finite params", sum(1 for p in vm.parameters() if not torch.isfinite(p).all()), flush=True)
        del vm, v
