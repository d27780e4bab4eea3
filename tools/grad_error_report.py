"""Numerical-error report used to set the GPU test bounds (tests/test_model_gpu.py,
tests/test_sampler_gpu.py): per-tensor relative Frobenius error ||a-b||/||b||
and max-abs error / max|b| of

1. the fused HIP program vs the same program on the PyTorch reference ops
   (identical bf16 rounding points: isolates kernel arithmetic / summation order),
2. the autograd wrapper (bf16 MFMA path) vs the plain fp32 PyTorch model,
3. the hipGraph DDIM sampler (k=20, N=64, 100 steps, fused head update) vs the
   fp32 eager loop from the same noise.

    python tools/grad_error_report.py  > gpurun_out/grad_error.txt
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from ddim_cold_amd import ops
from ddim_cold_amd.models import build_model
from ddim_cold_amd.models.program import ViTProgram, collect, model_tensors

DEV = "cuda"


def frob(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def mrel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / (b.abs().max() + 1e-30)).item()


def report(title, pairs):
    rows = sorted(((frob(a, b), mrel(a, b), n) for n, a, b in pairs), reverse=True)
    print(f"## {title}: worst frob {rows[0][0]:.3e} ({rows[0][2]}), worst max-rel "
          f"{max(r[1] for r in rows):.3e}; median frob {rows[len(rows) // 2][0]:.3e}", flush=True)
    for f, m, n in rows[:6]:
        print(f"   {n:40s} frob {f:.3e}  max-rel {m:.3e}")


def program_vs_ref_ops(name):
    torch.manual_seed(0)
    m = build_model(name).to(DEV).train()
    prog = ViTProgram.from_model(m)
    P = model_tensors(m)
    B = 8
    img = torch.randn(B, 3, 64, 64, device=DEV).clamp(-1, 1)
    tgt = torch.randn_like(img).clamp(-1, 1)
    t = torch.randint(0, 2000, (B,), device=DEV)
    r = torch.tensor([77, 3], dtype=torch.int64, device=DEV)
    res = []
    for force in (False, True):
        grads = {n: torch.zeros_like(p) for n, p in m.named_parameters()}
        G = collect(grads, prog.cfg.depth, prog.cfg.dim)
        ctx = ops.force_reference() if force else torch.no_grad()
        with ctx, torch.no_grad():
            out, S = prog.forward(P, img, t, r, True)
            loss, dtok = ops.smooth_l1_fwd_bwd(out, tgt, prog.cfg.tokens, prog.cfg.patch)
            prog.backward(P, G, S, dtok, r, True)
        torch.cuda.synchronize()
        res.append((out, grads))
    (o1, g1), (o2, g2) = res
    report(f"{name} program vs reference ops", [("out", o1, o2)] + [(n, g1[n], g2[n]) for n in g1])


def autograd_vs_fp32(name, depth=None, train=False, B=4, loss="square"):
    """Fused autograd path (bf16 MFMA kernels, hand-written backward) vs the plain fp32
    model's autograd (``forward_reference``), forward output and every gradient.
    ``train``: train mode with every dropout / drop-path probability 0 (the training
    kernels, no random masks)."""
    torch.manual_seed(0)
    kw = {} if depth is None else {"depth": depth}
    if train:
        kw.update(drop_rate=0.0, attn_drop_rate=0.0, drop_path_rate=0.0)
    m = build_model(name, **kw).to(DEV).train(train)
    H, W = m.img_size
    img = torch.randn(B, 3, H, W, device=DEV).clamp(-1, 1)
    tgt = torch.randn(B, 3, H, W, device=DEV).clamp(-1, 1)
    t = torch.randint(0, 2000, (B,), device=DEV)

    def lossf(o):
        return o.square().mean() if loss == "square" else torch.nn.functional.smooth_l1_loss(o, tgt)
    out = m(img, t)
    lossf(out).backward()
    g = {n: p.grad.clone() for n, p in m.named_parameters()}
    m.zero_grad()
    ref = m.forward_reference(img, t)
    lossf(ref).backward()
    tag = f"{name}{'' if depth is None else f' depth {depth}'} {'train p=0' if train else 'eval'} {loss}"
    report(f"{tag}: autograd (bf16 MFMA) vs fp32 model", [("out", out.detach(), ref.detach())] +
           [(n, g[n], p.grad) for n, p in m.named_parameters()])


def sampler_vs_eager(name="vit_tiny", k=20, N=64, depth=None):
    from ddim_cold_amd.bench.eager_sampler import eager_ddim_sample
    from ddim_cold_amd.diffusion.samplers import DDIMSampler
    torch.manual_seed(0)
    m = build_model(name, **({} if depth is None else {"depth": depth})).to(DEV).eval()
    H, W = m.img_size
    noise = torch.normal(0.0, 1.0, (N, 3, H, W), generator=torch.Generator().manual_seed(5))
    fused = DDIMSampler(m, DEV, k=k).sample(N, noise=noise)
    eager = eager_ddim_sample(m, DEV, k, N, noise=noise.to(DEV))
    d = (fused - eager).abs()
    print(f"## {name} sampler k={k} N={N} ({2000 // k} steps) fused vs eager fp32: mean |d| {d.mean():.3e}  "
          f"max |d| {d.max():.3e}  frob {frob(fused, eager):.3e}  (images in [0,1])", flush=True)


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    if which in ("all", "base"):
        for nm in ("vit_tiny", "oxford_flower"):
            program_vs_ref_ops(nm)
            autograd_vs_fp32(nm)
        sampler_vs_eager()
    if which in ("all", "r5"):
        # round 5: the fp32-oracle coverage of the non-yaml configs, train (p=0) and eval,
        # the smooth-L1 training loss; the flash path (626 tokens) at depth 2-3
        autograd_vs_fp32("oxford_flower", train=True, loss="smooth_l1")
        autograd_vs_fp32("oxford_flower", train=False, loss="smooth_l1")
        autograd_vs_fp32("vit_small_200", depth=3, train=True, B=2, loss="smooth_l1")
        autograd_vs_fp32("vit_small_200", depth=3, train=False, B=2, loss="smooth_l1")
        autograd_vs_fp32("vit_small_200", depth=2, train=True, B=2, loss="square")
        sampler_vs_eager("oxford_flower", k=20, N=16)
        sampler_vs_eager("vit_small_200", k=200, N=4, depth=3)
    if which in ("all", "r6"):
        # round 6: the benchmarked long-sequence sampler configuration at full depth
        # (vit_small_200, depth 12, 626 tokens, k=20 -> 100 steps), N=8, and the
        # ViT-tiny training gradients of the full model against the fp32 model
        sampler_vs_eager("vit_small_200", k=20, N=8)
        autograd_vs_fp32("vit_small_200", train=True, B=2, loss="smooth_l1")
