"""Graph-captured fused samplers on the GPU vs the plain eager PyTorch loop (fp32 reference
model + reference DDIM algebra), same initial noise."""
import math

import pytest
import torch

from ddim_cold_amd import build_model
from ddim_cold_amd.diffusion import schedule as sch
from ddim_cold_amd.diffusion.samplers import ColdSampler, DDIMSampler, img2img
from ddim_cold_amd.ops import reference as ref

DEV = "cuda"
# bounds on |fused - fp32 eager| of final images in [0, 1] after 100-200 DDIM steps
# (measured on MI355X, round 3, tools/grad_error_report.py: k=20 N=64 mean 7.9e-4,
# max 5.0e-3 -- the bf16 x0-hat error of each step is re-injected 100 times and
# amplified up to ~316x by x_t / sqrt(a_t) at t = 1999, so the max bound is looser)
MEAN_BOUND_K20 = 5e-3
MAX_BOUND_K20 = 0.1


@pytest.fixture(scope="module")
def model():
    torch.manual_seed(0)
    return build_model("vit_tiny").to(DEV).eval()


def _ref_ddim(model, noise, k):
    x = noise.to(DEV)
    with torch.no_grad():
        for t in sch.ddim_timesteps(model.total_steps, k):
            x0_raw = model.forward_reference(x, torch.full((x.shape[0],), t, device=DEV))
            x, x0 = ref.ddim_step(x, x0_raw, sch.ddim_coefficients(model.total_steps, t, k))
    return (x0.cpu() + 1) / 2


@pytest.mark.gpu
def test_ddim_sampler_matches_eager_reference(model):
    noise = torch.randn(8, 3, 64, 64, generator=torch.Generator().manual_seed(1))
    out = DDIMSampler(model, DEV, k=400).sample(8, noise=noise)
    exp = _ref_ddim(model, noise, 400)
    d = (out - exp).abs()
    assert d.mean() < 0.01 and d.max() < 0.2, (d.mean(), d.max())
    # graph replay reproduces the capture run
    out2 = DDIMSampler(model, DEV, k=400).sample(8, noise=noise)
    assert torch.equal(out, out2)
    seq = DDIMSampler(model, DEV, k=400).sequence(8, noise=noise)
    assert len(seq) == 6 and torch.allclose(seq[-1], out, atol=1e-6)


@pytest.mark.gpu
def test_cold_sampler_matches_eager_reference(model):
    s = ColdSampler(model, DEV)
    g = torch.Generator().manual_seed(2)
    init = s._init(4, g)
    seq = s.sequence(4, generator=torch.Generator().manual_seed(2))
    x = init.to(DEV)
    with torch.no_grad():
        for t in range(s.steps, 0, -1):
            x = model.forward_reference(x, torch.full((4,), t, device=DEV)).clamp(-1, 1)
    d = (seq[-1] - (x.cpu() + 1) / 2).abs()
    assert d.mean() < 0.01 and d.max() < 0.2, (d.mean(), d.max())


@pytest.mark.gpu
def test_ddim_sampler_benchmark_config_pinned(model):
    """The benchmarked configuration (k=20, N=64: 100 steps, x_t/sqrt(a_t) ~ 316x at
    t=1999) against the fp32 eager loop from the same noise.  The fused path runs
    bf16 MFMA GEMMs; the per-step x0-hat error (~1e-2 of the image range) is
    re-injected every step, so the bound is on the final images in [0, 1]."""
    noise = torch.randn(64, 3, 64, 64, generator=torch.Generator().manual_seed(7))
    out = DDIMSampler(model, DEV, k=20).sample(64, noise=noise)
    exp = _ref_ddim(model, noise, 20)
    d = (out - exp).abs()
    print(f"k=20 N=64: mean |d| {d.mean():.4f} max |d| {d.max():.4f}")
    assert d.mean() < MEAN_BOUND_K20 and d.max() < MAX_BOUND_K20, (d.mean(), d.max())


@pytest.mark.gpu
def test_img2img_gpu_batched(model):
    draft = torch.rand(3, 64, 64) * 2 - 1
    out = img2img(model, draft, [1199, 1599, 1999], k=400, device=DEV, generator=torch.Generator().manual_seed(3))
    assert out.shape == (3, 3, 64, 64) and torch.isfinite(out).all()
    assert out.min() >= 0 and out.max() <= 1


@pytest.mark.gpu
def test_img2img_graph_replay_matches_sequential_reference(model):
    """The draft->drawing configuration (ViT_draft2drawing.py:389-409: 9 t_starts
    1599..1999, k=10, up to 200 steps) as ONE batched, replayed hipGraph whose
    head epilogue applies per-sample DDIM coefficients: the replay reproduces the
    first (eager + capture) call bit for bit, each sample matches the reference's
    sequential batch-1 fp32 loop from the same noised input, and the replay is
    faster than that loop."""
    import time
    from ddim_cold_amd.bench.eager_sampler import eager_img2img
    from ddim_cold_amd.diffusion.samplers import ddim_from_starts, img2img_noised
    starts = list(range(1599, 2000, 50))
    g = torch.Generator().manual_seed(9)
    draft = (torch.rand(1, 3, 64, 64, generator=g) * 2 - 1).to(DEV)
    eps = torch.randn(len(starts), 3, 64, 64, generator=g).to(DEV)
    model.__dict__.pop("_sampler_graphs", None)
    x = img2img_noised(draft, eps, starts, model.total_steps)
    first = ddim_from_starts(model, x, starts, 10).clone()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    again = ddim_from_starts(model, x, starts, 10).clone()
    torch.cuda.synchronize()
    t_graph = time.perf_counter() - t0
    assert torch.equal(first, again)
    t0 = time.perf_counter()
    exp = eager_img2img(model, DEV, draft, starts, 10, eps)
    torch.cuda.synchronize()
    t_eager = time.perf_counter() - t0
    d = ((first - exp).abs() / 2)  # on the [0, 1] image scale
    print(f"img2img 9 starts k=10: graph {t_graph * 1e3:.2f} ms, eager {t_eager * 1e3:.1f} ms; "
          f"mean |d| {d.mean():.4f} max |d| {d.max():.4f}")
    assert d.mean() < MEAN_BOUND_K20 and d.max() < MAX_BOUND_K20, (d.mean(), d.max())
    assert t_graph < t_eager / 4, (t_graph, t_eager)


@pytest.mark.gpu
def test_patch_row_chain(model, monkeypatch):
    """Head epilogue -> next step's patch rows: the patch embedding without its patchify
    launch (cls rows from the GEMM epilogue) gives the same tokens, and the sampler
    with the chain matches the sampler without it."""
    from ddim_cold_amd import ops
    from ddim_cold_amd.diffusion import samplers as smp
    from ddim_cold_amd.models.program import model_tensors
    P = model_tensors(model)
    B, D = 6, model.embed_dim
    img = torch.randn(B, 3, 64, 64, device=DEV)
    t = torch.randint(0, 2000, (B,), device=DEV)
    r = torch.zeros(2, dtype=torch.int64, device=DEV)
    N = 65
    outs = []
    for chained in (False, True):
        st = torch.full((B * N, D // 32, 2), float("nan"), device=DEV)
        xb = torch.empty(B * N, D, dtype=torch.bfloat16, device=DEV)
        pin = None
        if chained:  # the bf16 patch rows a head epilogue would have written
            _, pin = ops.patch_embed_fwd(img, t, P.pe_w, P.pe_b, P.cls, P.pos, P.temb, r, 0, 0.0, 8)
        x, _ = ops.patch_embed_fwd(img, t, P.pe_w, P.pe_b, P.cls, P.pos, P.temb, r, 0, 0.0, 8, ln_st=st, xb_out=xb,
                                   patches_in=pin)
        outs.append((x.clone(), xb.clone(), st.sum(1)))
    (x1, xb1, s1), (x2, xb2, s2) = outs
    assert torch.equal(x1, x2) and torch.equal(xb1, xb2)
    assert torch.allclose(s1, s2, rtol=1e-5, atol=1e-4)  # per-slot partials vs one sum in slot 0
    noise = torch.randn(8, 3, 64, 64, generator=torch.Generator().manual_seed(4))
    res = []
    for on in (False, True):
        monkeypatch.setattr(smp, "PATCH_CHAIN", on)
        monkeypatch.setattr(smp, "ROWS", False)  # image-layout chain (rows: test_sampler_rows_gpu.py)
        model.__dict__.pop("_sampler_graphs", None)
        res.append(DDIMSampler(model, DEV, k=200).sample(8, noise=noise))
        res.append(ColdSampler(model, DEV).sequence(4, generator=torch.Generator().manual_seed(5))[-1])
    model.__dict__.pop("_sampler_graphs", None)
    assert (res[0] - res[2]).abs().max() < 1e-3
    assert (res[1] - res[3]).abs().max() < 1e-3
