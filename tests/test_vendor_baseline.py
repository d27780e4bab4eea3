"""The same-node vendor comparators (ddim_cold_amd/bench/vendor_baseline.py):
CPU plumbing checks of the code the GPU bench captures into one graph, and a
GPU run of both graphs."""
import math

import pytest
import torch

from ddim_cold_amd.bench.eager_sampler import eager_ddim_sample
from ddim_cold_amd.bench.vendor_baseline import (VendorSampler, VendorTrainStep, cold_batch_torch,
                                                 vendor_forward)
from ddim_cold_amd.models.vit import DiffusionVisionTransformer
from ddim_cold_amd.ops.reference import pixelate


def _tiny():
    torch.manual_seed(0)
    return DiffusionVisionTransformer(img_size=[16, 16], patch_size=4, embed_dim=32, depth=2, num_heads=4,
                                      total_steps=2000)


def test_sdpa_forward_matches_reference_eval():
    m = _tiny().eval()
    x = torch.randn(3, 3, 16, 16)
    t = torch.tensor([1, 500, 1999])
    with torch.no_grad():
        a = vendor_forward(m, x, t, "sdpa")
        b = m.forward_reference(x, t)
    torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5)


def test_cold_batch_torch_is_nearest_pixelation():
    torch.manual_seed(3)
    pool = torch.rand(10, 3, 64, 64) * 2 - 1
    x_t, x_tm1, t = cold_batch_torch(pool, 16, 6)
    assert t.min() >= 1 and t.max() <= 6
    for b in range(16):
        # identify the drawn image by its top-left pixel block at the finest level (t-1 >= 0)
        s = int(t[b])
        cand = [i for i in range(10) if torch.equal(pixelate(pool[i:i + 1], 2 ** (s - 1))[0], x_tm1[b])]
        assert cand, "x_{t-1} is not a NEAREST pixelation of a pool image"
        torch.testing.assert_close(x_t[b], pixelate(pool[cand[0]:cand[0] + 1], 2 ** s)[0], rtol=0, atol=0)


def test_gemm_bias_grad_and_mean_match_stock_ops():
    """_linear (bias gradient as a GEMM) and _mean (GEMV) == nn.Linear / .mean() gradients."""
    from ddim_cold_amd.bench.vendor_baseline import _linear, _mean
    torch.manual_seed(1)
    lin = torch.nn.Linear(24, 40)
    x = torch.randn(3, 7, 24, requires_grad=True)
    y1 = _mean(_linear(lin, x) ** 2)
    g1 = torch.autograd.grad(y1, [x, lin.weight, lin.bias])
    y2 = (lin(x) ** 2).mean()
    g2 = torch.autograd.grad(y2, [x, lin.weight, lin.bias])
    torch.testing.assert_close(y1, y2, rtol=1e-5, atol=1e-6)
    for a, b in zip(g1, g2):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def test_patch_gemm_matches_conv():
    """The comparator's GEMM patch embedding == nn.Conv2d (values and gradients)."""
    from ddim_cold_amd.bench.vendor_baseline import _patch_gemm
    m = _tiny()
    x = torch.randn(2, 3, 16, 16, requires_grad=True)
    a = _patch_gemm(m, x)
    b = m.patch_embed(x)
    torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5)
    ga = torch.autograd.grad(a.square().sum(), [x, m.patch_embed.proj.weight, m.patch_embed.proj.bias])
    gb = torch.autograd.grad(b.square().sum(), [x, m.patch_embed.proj.weight, m.patch_embed.proj.bias])
    for u, v in zip(ga, gb):
        torch.testing.assert_close(u, v, rtol=1e-4, atol=1e-5)


def test_vendor_train_step_cpu_runs_and_follows_cosine():
    m = _tiny()
    pool = torch.rand(8, 3, 16, 16) * 2 - 1
    before = [p.detach().clone() for p in m.parameters()]
    v = VendorTrainStep(m, pool, batch=4, lr=1e-3, t_max=10, use_graph=False)
    v.steps(3)
    assert math.isfinite(float(v.loss))
    assert float(v.step_t) == 3
    assert any(not torch.equal(a, b) for a, b in zip(before, m.parameters()))
    # lr used by the 3rd step = cosine at step index 2
    assert abs(v.opt.param_groups[0]["lr"] - 0.5e-3 * (1 + math.cos(math.pi * 2 / 10))) < 1e-12


def test_vendor_sampler_cpu_matches_eager_loop():
    m = _tiny().eval()
    s = VendorSampler(m, N=2, k=500, use_graph=False)
    g = torch.Generator().manual_seed(5)
    out = s.sample(g)
    ref = eager_ddim_sample(m, torch.device("cpu"), 500, 2, noise=s.x_in.clone())
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)
    assert s.ts == [1999, 1499, 999, 499]


def test_vendor_img2img_cpu_matches_sequential_reference_loop():
    """The batched vendor draft->drawing loop (all starts in one batch on the shared
    grid) == the reference's one-start-at-a-time loop (ViT_draft2drawing.py:394-409)."""
    from ddim_cold_amd.bench.eager_sampler import eager_img2img
    from ddim_cold_amd.bench.vendor_baseline import VendorImg2Img
    m = _tiny().eval()
    starts = [1599, 1649, 1699]
    v = VendorImg2Img(m, starts, k=50, use_graph=False)
    C, (H, W) = m.in_chans, m.img_size
    draft = torch.rand(1, C, H, W, generator=torch.Generator().manual_seed(2)) * 2 - 1
    out = v(draft, torch.Generator().manual_seed(7))
    eps = torch.normal(0.0, 1.0, (3, C, H, W), generator=torch.Generator().manual_seed(7))
    ref = eager_img2img(m, torch.device("cpu"), draft, starts, 50, eps)
    torch.testing.assert_close(out, (ref + 1) / 2, rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
def test_vendor_graphs_gpu():
    from ddim_cold_amd.bench.vendor_baseline import time_vendor_sampler, time_vendor_train
    from ddim_cold_amd.data.synthetic import synthetic_pool
    from ddim_cold_amd.models import build_model
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = build_model("vit_tiny").to(dev)
    pool = synthetic_pool(64, (64, 64), seed=1, device=dev)
    dt, loss, kind = time_vendor_train(m, pool, 32, 3.125e-4, 51200, steps=5, warmup=3)
    assert dt > 0 and math.isfinite(loss)
    # graph replay == eager body on the same model (one more step each; loss finite, params finite)
    assert all(torch.isfinite(p).all() for p in m.parameters())
    # back-to-back replays (no host sync between them): a valid smooth-L1 loss throughout
    v = VendorTrainStep(m, pool, 32, 3.125e-4, 51200)
    losses = []
    for _ in range(6):
        v.steps(10)
        losses.append(float(v.loss))
    assert all(0.0 <= l < 1.0 for l in losses), losses
    assert all(torch.isfinite(p).all() for p in m.parameters())
    # sampler graph == its eager loop on the same noise (2 DDIM steps)
    m.eval()
    sg = VendorSampler(m, 4, 1000)
    a = sg.sample(torch.Generator(device=dev).manual_seed(3))
    sg.use_graph = False
    b = sg.sample(torch.Generator(device=dev).manual_seed(3))
    torch.testing.assert_close(a, b, rtol=0, atol=2e-2)
    ts = time_vendor_sampler(m, 8, 200, reps=1)
    assert ts > 0
    s = VendorSampler(m, 4, 200)
    out = s.sample(torch.Generator(device=dev).manual_seed(1))
    assert out.shape == (4, 3, 64, 64) and torch.isfinite(out).all()
    assert out.min() >= 0 and out.max() <= 1
    from ddim_cold_amd.bench.vendor_baseline import time_vendor_img2img
    assert time_vendor_img2img(m, list(range(1599, 2000, 50)), 10, reps=1) > 0
