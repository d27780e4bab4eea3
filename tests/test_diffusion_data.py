"""Diffusion math, samplers and data semantics on CPU."""
import math
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from ddim_cold_amd import build_model
from ddim_cold_amd.data import datasets as ds
from ddim_cold_amd.data.synthetic import ColdBatcher, GaussianBatcher, synthetic_pool
from ddim_cold_amd.diffusion import schedule as sch
from ddim_cold_amd.diffusion.samplers import ColdSampler, DDIMSampler, img2img
from ddim_cold_amd.models import DiffusionVisionTransformer
from ddim_cold_amd.ops import reference as ref
from ddim_cold_amd import ops


# ----------------------------------------------------------------------------- schedule
def test_ddim_timesteps():
    assert sch.ddim_timesteps(2000, 20) == list(range(1999, 0, -20))
    assert len(sch.ddim_timesteps(2000, 20)) == 100
    assert sch.ddim_timesteps(2000, 400) == [1999, 1599, 1199, 799, 399]
    with pytest.raises(ValueError):
        sch.ddim_timesteps(2000, 300)  # last t=199, t+1-k < 0 (reference: math domain error)
    with pytest.raises(ValueError):
        sch.ddim_timesteps(2000, 0)


def test_ddim_coefficients_match_reference_formula():
    T, k = 2000, 20
    for t in [1999, 1000, 19]:
        a_t = 1 - math.sqrt((t + 1) / T) + 1e-5
        a_tk = 1 - math.sqrt((t + 1 - k) / T)
        c = sch.ddim_coefficients(T, t, k)
        assert c == pytest.approx((math.sqrt(a_t), math.sqrt(1 - a_t), math.sqrt(a_tk), math.sqrt(1 - a_tk)))
    assert sch.cold_steps(64) == 6 and sch.cold_steps(200) == 7
    assert sch.img2img_alpha(1000, 2000) == pytest.approx(1 - math.sqrt(0.5))


def test_ddim_step_identity():
    """x_{t-k} = sqrt(a_tk) x0 + sqrt(1-a_tk) * (x_t - sqrt(a_t) x0)/sqrt(1-a_t), x0 clamped."""
    torch.manual_seed(0)
    x = torch.randn(2, 3, 8, 8)
    x0 = torch.randn(2, 3, 8, 8) * 1.5
    coef = sch.ddim_coefficients(2000, 999, 20)
    xn, x0c = ref.ddim_step(x, x0, coef)
    c = x0.clamp(-1, 1)
    eps = (x - coef[0] * c) / coef[1]
    assert torch.allclose(xn, coef[2] * c + coef[3] * eps, atol=1e-6)
    assert torch.equal(x0c, c)
    # final step of a k | T grid: a_tk = 1 -> x_{t-k} == clamped x0
    cl = sch.ddim_coefficients(2000, 19, 20)
    assert cl[2] == 1.0 and cl[3] == 0.0
    xn, _ = ref.ddim_step(x, x0, cl)
    assert torch.allclose(xn, c)


def test_q_sample_statistics():
    x0 = torch.full((4096, 1, 1, 1), 0.5)
    eps = torch.randn(4096, 1, 1, 1, generator=torch.Generator().manual_seed(0))
    t = torch.full((4096,), 499)
    y = ref.q_sample(x0, t, eps, 2000)
    a = 1 - math.sqrt(500 / 2000)
    assert abs(y.mean().item() - math.sqrt(a) * 0.5) < 0.03
    assert abs(y.std().item() - math.sqrt(1 - a)) < 0.03


# ----------------------------------------------------------------------------- pixelation
@pytest.mark.parametrize("size,f", [(64, 2), (64, 8), (64, 64), (32, 4), (200, 8), (200, 64), (200, 128)])
def test_pixelate_matches_pil_nearest_semantics(size, f):
    """torch 'nearest' down to floor(W/f) then back up == floor-index gather (PIL NEAREST analogue)."""
    img = torch.randn(2, 3, size, size)
    ts = max(size // f, 1)
    src_small = (torch.arange(ts) * size / ts).floor().long()
    small = img[:, :, src_small][:, :, :, src_small]
    src_big = (torch.arange(size) * ts / size).floor().long()
    expect = small[:, :, src_big][:, :, :, src_big]
    assert torch.equal(ref.pixelate(img, f), expect)


def test_cold_dataset_pairs(tmp_path):
    from PIL import Image
    rng = np.random.default_rng(0)
    for i in range(3):
        Image.fromarray(rng.integers(0, 255, (40, 48, 3), dtype=np.uint8)).save(tmp_path / f"im{i}.png")
    (tmp_path / "notes.txt").write_text("skip me")
    d = ds.ColdDownSampleDataset(str(tmp_path), imgSize=(32, 32))
    assert len(d) == 3 and d.max_step == 5
    x_t, x_tm1, t = d.__getitem__(0, t=3)
    img = d._img(0)
    assert img.shape == (3, 32, 32) and img.min() >= -1 and img.max() <= 1
    assert torch.equal(x_t, ref.pixelate(img[None], 8)[0]) and torch.equal(x_tm1, ref.pixelate(img[None], 4)[0])
    for _ in range(20):
        _, _, t = d[1]
        assert 1 <= t <= 5
    xa, x0, t = ds.ColdDownSampleDataset_au(str(tmp_path), imgSize=(32, 32)).__getitem__(2, t=1)
    assert torch.equal(x0, d._img(2))
    xg, x0g, tg = ds.DiffusionDataset(str(tmp_path), imgSize=(32, 32)).__getitem__(0, t=0)
    assert xg.shape == x0g.shape == (3, 32, 32) and tg == 0
    cache = ds.DeviceImageCache(str(tmp_path), (32, 32), "cpu", workers=2)
    assert len(cache) == 3
    assert (cache.float_pool()[0] - img).abs().max() < 1e-6


@pytest.mark.parametrize("n,world,drop_last", [(100, 2, True), (101, 4, True), (101, 4, False), (7, 8, False)])
def test_shard_indices_match_distributed_sampler(n, world, drop_last):
    from torch.utils.data import DistributedSampler
    data = list(range(n))
    for epoch in [0, 3]:
        for r in range(world):
            s = DistributedSampler(data, num_replicas=world, rank=r, shuffle=True, seed=42, drop_last=drop_last)
            s.set_epoch(epoch)
            assert ds.shard_indices(n, world, r, epoch, 42, True, drop_last).tolist() == list(iter(s))


def test_cold_batcher_cpu_semantics():
    pool = synthetic_pool(16, size=(32, 32))
    assert pool.shape == (16, 3, 32, 32) and pool.min() >= -1 and pool.max() <= 1
    rng = torch.tensor([7, 0])
    b = ColdBatcher(pool, 8, rng)
    x_t, x_tm1, t = b()
    assert t.min() >= 1 and t.max() <= 5
    for i in range(8):
        img = pool[b.idx[i]][None]
        assert torch.equal(x_t[i], ref.pixelate(img, 2 ** int(t[i]))[0])
        assert torch.equal(x_tm1[i], ref.pixelate(img, 2 ** (int(t[i]) - 1))[0])
    # fixed index table (DistributedSampler order)
    idx = torch.arange(8)
    b2 = ColdBatcher(pool, 8, rng, idx=idx, target="x0")
    x_t, x0, t = b2()
    assert torch.equal(x0, pool[:8])
    g = GaussianBatcher(pool, 8, rng)
    xg, x0g, tg = g()
    assert xg.shape == (8, 3, 32, 32) and tg.min() >= 0 and tg.max() < 2000
    # x_t = q_sample(x0, t, eps) with eps = randn_ at the noise site, x0 = pool[idx]
    from ddim_cold_amd import ops
    from ddim_cold_amd.data.synthetic import SITE_NOISE
    assert torch.equal(x0g, pool[g.idx])
    eps = torch.empty_like(xg)
    ops.randn_(eps, rng, SITE_NOISE)
    a = (1 - torch.sqrt((tg.double() + 1) / 2000)).float().view(-1, 1, 1, 1)
    assert torch.allclose(xg, a.sqrt() * x0g + (1 - a).sqrt() * eps, atol=1e-6)
    # the fused-spec form (patch-embedding launch) draws the same batch
    (xs, x0s, ts), spec = g.fused_spec()
    assert spec[8] == 2000 and spec[4] is True and xs is g.x_t and x0s is g.x0 and ts is g.t


def test_counter_rng_advances():
    rng = torch.tensor([7, 0])
    a = ref.keep_mask(10000, rng, 5, 0.1)
    assert abs(1 - a.float().mean().item() - 0.1) < 0.01
    assert torch.equal(a, ref.keep_mask(10000, rng, 5, 0.1))
    assert not torch.equal(a, ref.keep_mask(10000, rng, 6, 0.1))
    assert not torch.equal(a, ref.keep_mask(10000, torch.tensor([7, 1]), 5, 0.1))


@pytest.mark.parametrize("p", [0.1, 0.5])
def test_drop_mix_statistics(p):
    """The 24-bit-multiplier dropout hash (csrc/common.h drop_mix): drop rate, the two
    halves of one pair hash, neighbouring pairs and attention rows (stride ld) are
    independent within sampling noise (2^21 elements, 3 sigma)."""
    n = 1 << 21
    for step in (0, 1, 12345):
        k = ref.keep_mask(n, torch.tensor([20240521, step]), 3, p).float()
        sig = (p * (1 - p) / n) ** 0.5
        assert abs(1 - k.mean().item() - p) < 4 * sig
        even, odd = k[0::2], k[1::2]
        for a, b in ((even, odd), (odd[:-1], even[1:]), (k[:-640], k[640:]), (k[:-2], k[2:])):
            c = torch.corrcoef(torch.stack([a, b]))[0, 1].item()
            assert abs(c) < 4 / (a.numel() ** 0.5), c
    assert ref.drop_threshold(0.1) == 6554 and ref.drop_threshold(1.0) == 65536 and ref.drop_threshold(0.0) == 0


# ----------------------------------------------------------------------------- samplers (CPU reference path)
@pytest.fixture(scope="module")
def tiny():
    torch.manual_seed(0)
    return DiffusionVisionTransformer(img_size=[16, 16], patch_size=4, embed_dim=32, depth=1, num_heads=2).eval()


def test_ddim_sampler_matches_manual_loop(tiny):
    noise = torch.randn(2, 3, 16, 16)
    s = DDIMSampler(tiny, "cpu", k=400)
    out = s.sample(2, noise=noise)
    x = noise.clone()
    with torch.no_grad():
        for t in [1999, 1599, 1199, 799, 399]:
            x0 = tiny.forward_reference(x, torch.full((2,), t))
            x, x0c = ref.ddim_step(x, x0, sch.ddim_coefficients(2000, t, 400))
    assert torch.allclose(out, (x0c + 1) / 2, atol=1e-5)
    seq = s.sequence(2, noise=noise)
    assert len(seq) == 6 and torch.allclose(seq[-1], out, atol=1e-5)
    assert torch.allclose(seq[0], (noise + 1) / 2)


def test_model_sampler_api(tiny):
    g = torch.Generator().manual_seed(0)
    assert tiny.sampler("cpu", k=400, N=3, generator=g).shape == (3, 3, 16, 16)
    assert len(tiny.diffusion_sequence("cpu", k=400, N=2)) == 6
    assert tiny.cold_sampler("cpu", N=2).shape == (2, 3, 16, 16)
    assert len(tiny.cold_diffusion_sequence("cpu", N=2)) == sch.cold_steps(16) + 1


def test_cold_sampler(tiny):
    s = ColdSampler(tiny, "cpu")
    assert s.steps == 4
    seq = s.sequence(2, generator=torch.Generator().manual_seed(1))
    assert len(seq) == 5
    first = seq[0]
    assert torch.allclose(first, first[:, :, :1, :1].expand_as(first))  # constant-colour start
    assert seq[-1].min() >= 0 and seq[-1].max() <= 1


def test_img2img_batched_equals_sequential(tiny):
    draft = torch.rand(3, 16, 16) * 2 - 1
    starts = [1199, 1599, 1999]
    eps = torch.randn(3, 3, 16, 16, generator=torch.Generator().manual_seed(3))
    out = img2img(tiny, draft, starts, k=400, device="cpu", generator=torch.Generator().manual_seed(3))
    with torch.no_grad():
        for i, s in enumerate(starts):
            a = sch.img2img_alpha(s, 2000)
            x = math.sqrt(1 - a) * eps[i:i + 1] + math.sqrt(a) * draft[None]
            for t in range(s, 0, -400):
                x0 = tiny.forward_reference(x, torch.full((1,), t))
                x, x0c = ref.ddim_step(x, x0, sch.ddim_coefficients(2000, t, 400))
            assert torch.allclose(out[i], ((x0c + 1) / 2)[0], atol=1e-5), s


def test_starts_table_identity_rows_and_cache(tiny):
    """img2img's per-sample coefficient table: a sample joins the grid at its start step
    and carries the exact identity row {0, 1, 0, 1} before it; repeated calls reuse
    the cached loop state and reproduce the result."""
    from ddim_cold_amd.diffusion.samplers import ddim_from_starts, starts_table
    ts, coef = starts_table(2000, [1199, 1599, 1999], 400)
    assert ts == [1999, 1599, 1199, 799, 399]
    assert coef.shape == (5, 3, 4)
    assert coef[0, 0].tolist() == [0.0, 1.0, 0.0, 1.0] and coef[1, 0].tolist() == [0.0, 1.0, 0.0, 1.0]
    assert torch.allclose(coef[2, 0], torch.tensor(sch.ddim_coefficients(2000, 1199, 400)))
    assert torch.allclose(coef[0, 2], torch.tensor(sch.ddim_coefficients(2000, 1999, 400)))
    with pytest.raises(ValueError):
        starts_table(2000, [1999, 1998], 10)
    x = torch.randn(3, 3, 16, 16, generator=torch.Generator().manual_seed(4))
    a = ddim_from_starts(tiny, x, [1199, 1599, 1999], 400).clone()
    b = ddim_from_starts(tiny, x, [1199, 1599, 1999], 400).clone()
    assert torch.equal(a, b)
    assert sum(1 for k in tiny.__dict__["_sampler_graphs"] if k[0] == "img2img") == 1


def test_ddim_from_starts_result_not_aliased_and_cache_capped(tiny):
    """The returned x0-hat is the caller's own tensor (a later call with the same key
    does not overwrite it), and at most IMG2IMG_GRAPHS img2img loops stay cached."""
    from ddim_cold_amd.diffusion import samplers as smp
    x1 = torch.randn(2, 3, 16, 16, generator=torch.Generator().manual_seed(5))
    x2 = torch.randn(2, 3, 16, 16, generator=torch.Generator().manual_seed(6))
    a = smp.ddim_from_starts(tiny, x1, [1599, 1999], 400)
    a_copy = a.clone()
    b = smp.ddim_from_starts(tiny, x2, [1599, 1999], 400)
    assert torch.equal(a, a_copy) and not torch.equal(a, b)
    for i in range(smp.IMG2IMG_GRAPHS + 3):  # distinct keys
        smp.ddim_from_starts(tiny, x1, [1999 - 100 * i, 1999], 100)
    n = sum(1 for k in tiny.__dict__["_sampler_graphs"] if k[0] == "img2img")
    assert n <= smp.IMG2IMG_GRAPHS


def test_slerp_and_interpolate(tiny):
    from ddim_cold_amd.diffusion.interpolate import interpolate, slerp
    a, b = torch.randn(1, 3, 4, 4), torch.randn(1, 3, 4, 4)
    lam = torch.tensor([0.0, 0.5, 1.0])
    s = slerp(a, b, lam)
    assert torch.allclose(s[0], b[0], atol=1e-5) and torch.allclose(s[2], a[0], atol=1e-5)
    img1, img2 = torch.rand(3, 16, 16) * 2 - 1, torch.rand(3, 16, 16) * 2 - 1
    out = interpolate(tiny, img1, img2, t_starts=[399, 799], k=400, lambdas=torch.linspace(0, 1, 3), device="cpu",
                      generator=torch.Generator().manual_seed(0))
    assert out.shape == (3, 3, 3, 16, 16)
    assert torch.allclose(out[0, 0], (img1 + 1) / 2) and torch.allclose(out[0, 2], (img2 + 1) / 2)
    assert out.min() >= 0 and out.max() <= 1


def test_stepped_index_table_cpu():
    """Batch rows from a [rows, micro, B] table at the device step counter (the trainer's
    K-step-graph batch source) == the explicit [B] index row."""
    from ddim_cold_amd import ops
    from ddim_cold_amd.data.synthetic import make_batcher
    pool = synthetic_pool(24, size=(16, 16))
    table = torch.randperm(24)[:18].reshape(3, 2, 3)
    ctr = torch.tensor([0, 5])
    rng = torch.tensor([7, 2])
    for kind in ("cold", "cold_x0", "gaussian"):
        for j in range(2):
            want = table[5 % 3, j]
            assert torch.equal(ops.stepped_idx(table, (ctr[1:], 3 * j), 3), want)
            a = make_batcher(kind, pool, 3, rng, idx=table, idx_step=(ctr[1:], 3 * j))()
            b = make_batcher(kind, pool, 3, rng, idx=want.clone())()
            assert all(torch.equal(u, v) for u, v in zip(a, b)), kind
