"""Why the vendor comparator (ddim_cold_amd/bench/vendor_baseline.py) computes its bias
gradients and loss mean with GEMMs: an ATen multi-workgroup reduction captured in a
torch.cuda.CUDAGraph, replayed on changing input, vs the same sum eagerly and as a
GEMV; then the vendor training step's loss, graph vs eager, and the vendor DDIM
sampler graph vs its eager loop on the same noise (PyTorch 2.10 / ROCm 7, MI355X)."""
import sys

import torch

sys.path.insert(0, ".")
import ddim_cold_amd.bench.vendor_baseline as vb  # noqa: E402
from ddim_cold_amd.data.synthetic import synthetic_pool  # noqa: E402
from ddim_cold_amd.models import build_model  # noqa: E402

dev = torch.device("cuda", 0)

# 1. one global reduction in a graph
x = torch.randn(1 << 20, device=dev)
out = torch.zeros(2, device=dev)
ones = torch.ones(x.numel(), 1, device=dev)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    out[0].copy_(x.sum())
    out[1].copy_((x.view(1, -1) @ ones).reshape(()))
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    out[0].copy_(x.sum())
    out[1].copy_((x.view(1, -1) @ ones).reshape(()))
for i in range(4):
    x.normal_()
    g.replay()
    torch.cuda.synchronize()
    ref = float(x.double().cpu().sum())
    print(f"replay {i}: eager sum {ref:.3f}  graph x.sum() {float(out[0]):.3f}  graph GEMV {float(out[1]):.3f}",
          flush=True)

# 2. vendor training step: graph vs eager loss trajectory
MODEL = sys.argv[1] if len(sys.argv) > 1 else "vit_tiny"
pool = synthetic_pool(1024, (64, 64), seed=7, device=dev)
for graph in (False, True):
    torch.manual_seed(1234)
    m = build_model(MODEL).to(dev).train()
    st = vb.VendorTrainStep(m, pool, 32, 3.125e-4, 51200, use_graph=graph)
    trace = []
    for i in range(300):
        st.steps(1)
        if (i + 1) % 25 == 0:
            trace.append(round(float(st.loss), 4))
    nonfinite = sum(1 for p in m.parameters() if not torch.isfinite(p).all())
    print(f"{MODEL} vendor step {'graph' if graph else 'eager'}: loss every 25 steps {trace}; "
          f"non-finite params {nonfinite}",
          flush=True)

# 3. vendor sampler: graph vs eager on the same x_T
m.eval()
smp = vb.VendorSampler(m, 16, 20)
gen = torch.Generator(device=dev).manual_seed(5)
a = smp.sample(gen)
smp.use_graph = False
gen = torch.Generator(device=dev).manual_seed(5)
b = smp.sample(gen)
print(f"vendor sampler graph vs eager: max |diff| {float((a - b).abs().max()):.2e}, "
      f"mean {float(a.mean()):.4f} / {float(b.mean()):.4f}", flush=True)
