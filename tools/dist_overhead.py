"""Host vs device time per step of the segmented (multi-rank) engine path on ONE GPU (1-rank RCCL group)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.distributed as dist
os.environ.setdefault("MASTER_ADDR", "127.0.0.1"); os.environ.setdefault("MASTER_PORT", "29533")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
from ddim_cold_amd.models import build_model
from ddim_cold_amd.train.engine import EngineConfig, TrainEngine
from ddim_cold_amd.data.synthetic import ColdBatcher, synthetic_pool
bb = int(os.environ.get("BB", "2"))
model = build_model("vit_tiny").cuda().train()
eng = TrainEngine(model, EngineConfig(lr=1e-4, t_max=1000, force_segments=True, bucket_blocks=bb, temb_rows=7))
eng.set_batch_fn(ColdBatcher(synthetic_pool(256, device="cuda"), 32, eng.rng))
for _ in range(20):
    eng.train_step()
torch.cuda.synchronize()
n = 200
t0 = time.perf_counter()
for _ in range(n):
    eng.train_step()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
# per-call host costs
g = eng._graphs[0]
torch.cuda.synchronize(); a = time.perf_counter()
for _ in range(100): g.replay()
b = time.perf_counter(); torch.cuda.synchronize()
v = eng.flat_g[:1000000]
c = time.perf_counter()
for _ in range(100): dist.all_reduce(v)
d = time.perf_counter(); torch.cuda.synchronize()
print(f"BB={bb} segments={len(eng._graphs)} host/step {1e3*(t1-t0)/n:.3f} ms, device/step {1e3*(t2-t0)/n:.3f} ms; "
      f"replay host {1e6*(b-a)/100:.1f} us, all_reduce host {1e6*(d-c)/100:.1f} us")
dist.destroy_process_group()
