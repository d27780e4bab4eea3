"""Why the vendor comparator (ddim_cold_amd/bench/vendor_baseline.py) is written the way it
is, as GPU checks on PyTorch 2.10 / ROCm 7 (MI355X):

  reductions  an ATen global reduction captured in a graph vs a GEMV, replayed on changing
              input; then the vendor training step's loss, graph vs eager, over 300 replays
              (the Linear bias gradients and the loss mean are GEMMs: _AddBias / _mean)
  replay      back-to-back graph replays vs a host sync per replay, per model and attention
              core, on device memory pre-filled with NaN (an unwritten read turns NaN)
  patch       oxford_flower (p=4) with the MIOpen convolution vs the GEMM patch embedding
              (_patch_gemm), back to back and with a sync per replay
  sampler     the vendor DDIM sampler graph vs its eager loop on the same x_T

usage: python tools/vendor_debug.py [reductions|replay|patch|sampler ...] (default: all)"""
import sys

import torch

sys.path.insert(0, ".")
import ddim_cold_amd.bench.vendor_baseline as vb  # noqa: E402
from ddim_cold_amd.data.synthetic import synthetic_pool  # noqa: E402
from ddim_cold_amd.models import build_model  # noqa: E402

dev = torch.device("cuda", 0)
POOL = None


def pool():
    global POOL
    if POOL is None:
        POOL = synthetic_pool(1024, (64, 64), seed=7, device=dev)
    return POOL


def step(name, patch="gemm", attn="sdpa"):
    torch.manual_seed(1234)
    m = build_model(name).to(dev).train()
    return m, vb.VendorTrainStep(m, pool(), 32, 3.125e-4, 51200, attn=attn, patch=patch)


def nonfinite(m):
    return sum(1 for p in m.parameters() if not torch.isfinite(p).all())


def reductions():
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
        print(f"replay {i}: eager sum {float(x.double().cpu().sum()):.3f}  graph x.sum() {float(out[0]):.3f}  "
              f"graph GEMV {float(out[1]):.3f}", flush=True)
    for graph in (False, True):
        m, st = step("vit_tiny")
        st.use_graph = graph
        trace = []
        for i in range(300):
            st.steps(1)
            if (i + 1) % 25 == 0:
                trace.append(round(float(st.loss), 4))
        print(f"vit_tiny vendor step {'graph' if graph else 'eager'}: loss every 25 steps {trace}; "
              f"non-finite params {nonfinite(m)}", flush=True)


def pollute(gib=8):
    x = torch.full((gib << 28,), float("nan"), device=dev)
    del x
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def replay():
    for name in ("oxford_flower", "vit_tiny"):
        for attn in ("sdpa", "explicit"):
            for chunk in (1, 220):
                pollute()
                m, st = step(name, attn=attn)
                done, trace = 0, []
                while done < 220:
                    st.steps(chunk)
                    done += chunk
                    if done % 44 == 0 or chunk > 1:
                        trace.append(round(float(st.loss), 4))
                print(f"{name} attn={attn} replays per host sync={chunk}: loss {trace} "
                      f"non-finite params {nonfinite(m)}", flush=True)


def patch():
    for p in ("conv", "gemm"):
        for sync in (False, True):
            m, v = step("oxford_flower", patch=p)
            for _ in range(220):
                v.steps(1)
                if sync:
                    torch.cuda.synchronize()
            print(f"oxford_flower patch={p} {'sync every replay' if sync else 'back to back'}: loss "
                  f"{float(v.loss):.5f} non-finite params {nonfinite(m)}", flush=True)


def sampler():
    torch.manual_seed(0)
    m = build_model("vit_tiny").to(dev).eval()
    smp = vb.VendorSampler(m, 16, 1000)
    a = smp.sample(torch.Generator(device=dev).manual_seed(5))
    smp.use_graph = False
    b = smp.sample(torch.Generator(device=dev).manual_seed(5))
    print(f"vendor sampler graph vs eager: max |diff| {float((a - b).abs().max()):.2e}", flush=True)


CHECKS = {"reductions": reductions, "replay": replay, "patch": patch, "sampler": sampler}
for c in (sys.argv[1:] or list(CHECKS)):
    CHECKS[c]()
