"""Vendor training step: back-to-back graph replays (no host sync) vs one sync per replay, per model
and attention core -- a replay-order hazard shows as a NaN only in the back-to-back runs."""
import sys
import torch
sys.path.insert(0, ".")
import ddim_cold_amd.bench.vendor_baseline as vb
from ddim_cold_amd.data.synthetic import synthetic_pool
from ddim_cold_amd.models import build_model
dev = torch.device("cuda", 0)
pool = synthetic_pool(1024, (64, 64), seed=7, device=dev)


def pollute(gib=8):
    """Device memory handed back to the driver full of NaN bit patterns, so a kernel that
    reads memory it never wrote (a stale reduction output, an unzeroed workspace) turns NaN."""
    x = torch.full((gib << 28,), float("nan"), device=dev)
    del x
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


for name in ("oxford_flower", "vit_tiny"):
    for attn in ("sdpa", "explicit"):
        for chunk in (1, 220):
            pollute()
            torch.manual_seed(1234)
            m = build_model(name).to(dev).train()
            st = vb.VendorTrainStep(m, pool, 32, 3.125e-4, 51200, attn=attn)
            done, trace = 0, []
            while done < 220:
                st.steps(chunk)
                done += chunk
                if done % 44 == 0 or chunk > 1:
                    trace.append(round(float(st.loss), 4))
            bad = sum(1 for p in m.parameters() if not torch.isfinite(p).all())
            print(f"{name} attn={attn} replays per host sync={chunk}: loss {trace} non-finite params {bad}", flush=True)
