"""Why the vendor comparator's dropout is a mask multiply (ddim_cold_amd/bench/vendor_baseline._drop):
per-replay loss of the graph-captured bf16-autocast vendor training step with native
``F.dropout`` (NaN after ~12 replays on PyTorch 2.10 / ROCm 7, MI355X) vs the mask form."""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
import ddim_cold_amd.bench.vendor_baseline as vb  # noqa: E402
from ddim_cold_amd.data.synthetic import synthetic_pool  # noqa: E402
from ddim_cold_amd.models import build_model  # noqa: E402

dev = torch.device("cuda", 0)
pool = synthetic_pool(1024, (64, 64), seed=7, device=dev)
mask_drop = vb._drop
for name, fn in (("native F.dropout", lambda x, p, tr: F.dropout(x, p, True) if tr and p > 0 else x),
                 ("mask", mask_drop)):
    vb._drop = fn
    torch.manual_seed(1234)
    m = build_model("vit_tiny").to(dev).train()
    v = vb.VendorTrainStep(m, pool, 32, 3.125e-4, 51200, use_graph=True)
    trace = []
    for _ in range(30):
        v.steps(1)
        torch.cuda.synchronize()
        trace.append(round(float(v.loss), 4))
    print(name, trace, "non-finite params:", sum(1 for p in m.parameters() if not torch.isfinite(p).all()),
          flush=True)
vb._drop = mask_drop
