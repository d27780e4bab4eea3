"""Scratch timing: torch-eager reference step vs fused HIP program (eager and graph)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from ddim_cold_amd.models import build_model
from ddim_cold_amd.models.program import ViTProgram, collect, model_tensors
from ddim_cold_amd import ops

dev = "cuda"
B = int(os.environ.get("B", 32))
torch.manual_seed(0)
m = build_model("vit_tiny").to(dev).train()
img = torch.randn(B, 3, 64, 64, device=dev).clamp(-1, 1)
tgt = torch.randn_like(img).clamp(-1, 1)
t = torch.randint(1, 7, (B,), device=dev)

def timeit(fn, n=30, w=5):
    for _ in range(w): fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n): fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3

# 1) torch eager reference (autocast bf16 + AdamW + clip)
opt = torch.optim.AdamW(m.parameters(), lr=1e-4, weight_decay=0.05)
def ref_step():
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = m.forward_reference(img, t)
        loss = torch.nn.functional.smooth_l1_loss(out.float(), tgt)
    opt.zero_grad(set_to_none=False)
    loss.backward()
    torch.nn.utils.clip_grad_norm_(m.parameters(), 1.0)
    opt.step()
ms = timeit(ref_step)
print(f"torch eager reference step: {ms:.3f} ms  -> {B/ms*1e3:.0f} img/s", flush=True)

# 2) fused program fwd+bwd (eager launches)
prog = ViTProgram.from_model(m)
P = model_tensors(m)
grads = {n: torch.zeros_like(p) for n, p in m.named_parameters()}
G = collect(grads, prog.cfg.depth, prog.cfg.dim)
r = torch.tensor([1, 0], dtype=torch.int64, device=dev)
def fused_step():
    out, S = prog.forward(P, img, t, r, True)
    loss, dtok = ops.smooth_l1_fwd_bwd(out, tgt, prog.cfg.tokens, prog.cfg.patch)
    prog.backward(P, G, S, dtok, r, True)
    return loss
with torch.no_grad():
    ms = timeit(fused_step)
    print(f"fused fwd+bwd eager: {ms:.3f} ms -> {B/ms*1e3:.0f} img/s", flush=True)
    # 3) graph captured
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3): fused_step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fused_step()
    ms = timeit(g.replay, n=100, w=10)
print(f"fused fwd+bwd graph: {ms:.3f} ms -> {B/ms*1e3:.0f} img/s", flush=True)
