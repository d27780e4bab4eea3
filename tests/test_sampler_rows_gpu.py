"""Patch-row sampler state (ops.head_step_rows_, EPI_HEADR vector epilogue) vs the
image-layout head step: same math per element, contiguous accesses."""
import pytest
import torch

from ddim_cold_amd import build_model, ops
from ddim_cold_amd.diffusion import samplers

DEV = "cuda"


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2, 4])
def test_head_step_rows_matches_image_layout(mode):
    torch.manual_seed(0)
    B, C, H, W, p, D = 6, 3, 64, 64, 8, 384
    NP, F = (H // p) * (W // p), C * p * p
    M = B * (NP + 1)
    a = torch.randn(M, D, device=DEV).to(torch.bfloat16)
    st = torch.empty(M, D // 32, 2, device=DEV)
    xa = a.float().view(M, D // 32, 32)
    st[..., 0], st[..., 1] = xa.sum(-1), (xa * xa).sum(-1)
    w = (torch.randn(F, D, device=DEV) * 0.05).to(torch.bfloat16)
    b = torch.randn(F, device=DEV) * 0.1
    c = w.float().sum(1)
    fold = (st, c, 1e-5)
    x = torch.randn(B, C, H, W, device=DEV)
    x0 = torch.zeros_like(x)
    coef = torch.tensor([0.3, 0.95, 0.5, 0.86], device=DEV) if mode != 4 else \
        torch.rand(B, 4, device=DEV) * 0.5 + 0.5
    pout = torch.zeros(B * NP, F, dtype=torch.bfloat16, device=DEV)
    xr = ops.image_to_rows(x, p).contiguous()
    x0r = torch.zeros_like(xr)
    pr = torch.zeros_like(pout)
    ops.head_step_(a, w, b, x, x0, coef, p, mode, fold=fold, patches_out=pout)
    ops.head_step_rows_(a, w, b, xr, x0r, coef, B, mode, fold=fold, patches_out=pr)
    torch.cuda.synchronize()
    assert (ops.image_to_rows(x, p) - xr).abs().max().item() < 1e-4
    if mode != 2:
        assert (ops.image_to_rows(x0, p) - x0r).abs().max().item() < 1e-5
    # the image-layout chain writes conv-order patch rows; the rows chain head order
    assert torch.equal(pr.float(), xr.to(torch.bfloat16).float())
    conv = x.reshape(B, C, H // p, p, W // p, p).permute(0, 2, 4, 1, 3, 5).reshape(B * NP, F)
    assert (pout.float() - conv.to(torch.bfloat16).float()).abs().max().item() <= 1e-2


@pytest.mark.gpu
def test_rows_sampler_matches_image_layout_sampler():
    torch.manual_seed(0)
    model = build_model("vit_tiny").to(DEV).eval()
    noise = torch.randn(8, 3, 64, 64, generator=torch.Generator().manual_seed(3))
    outs = {}
    for rows in (True, False):
        samplers.ROWS = rows
        model.__dict__.pop("_sampler_graphs", None)
        try:
            d = samplers.DDIMSampler(model, DEV, k=100).sample(8, noise=noise)
            d2 = samplers.DDIMSampler(model, DEV, k=100).sample(8, noise=noise)  # replay
            assert torch.equal(d, d2)
            seq = samplers.DDIMSampler(model, DEV, k=100).sequence(8, noise=noise)
            cs = samplers.ColdSampler(model, DEV).sequence(4, generator=torch.Generator().manual_seed(2))
            ii = samplers.img2img(model, noise[0], [1599, 1799, 1999], 100,
                                  generator=torch.Generator().manual_seed(4))
            outs[rows] = (d, seq, cs, ii)
        finally:
            samplers.ROWS = True
            model.__dict__.pop("_sampler_graphs", None)
    (d1, s1, c1, i1), (d0, s0, c0, i0) = outs[True], outs[False]
    assert (d1 - d0).abs().mean() < 2e-3 and (d1 - d0).abs().max() < 0.05
    assert len(s1) == len(s0) and torch.allclose(s1[-1], d1, atol=1e-6)
    assert all((a - b).abs().mean() < 2e-3 for a, b in zip(s1, s0))
    assert len(c1) == len(c0) and all((a - b).abs().max() < 2e-2 for a, b in zip(c1, c0))
    assert (i1 - i0).abs().mean() < 2e-3


@pytest.mark.gpu
def test_head_loss_rows_matches_image_layout():
    """Training loss epilogue on a patch-row target (EPI_HEADL) == the image-layout one."""
    torch.manual_seed(1)
    B, C, H, W, p, D = 32, 3, 64, 64, 8, 384
    NP, F = (H // p) * (W // p), C * p * p
    M = B * (NP + 1)
    a = torch.randn(M, D, device=DEV).to(torch.bfloat16)
    st = torch.empty(M, D // 32, 2, device=DEV)
    xa = a.float().view(M, D // 32, 32)
    st[..., 0], st[..., 1] = xa.sum(-1), (xa * xa).sum(-1)
    w = (torch.randn(F, D, device=DEV) * 0.05).to(torch.bfloat16)
    b = torch.randn(F, device=DEV) * 0.1
    c = w.float().sum(1)
    tgt = torch.randn(B, C, H, W, device=DEV).clamp(-1, 1)
    m0, r0, m1, r1 = (torch.empty(M, device=DEV) for _ in range(4))
    parts0, g0 = ops.head_loss(a, w, b, tgt, p, 1.0, fold=(st, c, 1e-5, m0, r0))
    rows = ops.image_to_rows(tgt, p).contiguous().view(B, C, H, W)
    parts1, g1 = ops.head_loss(a, w, b, rows, p, 1.0, fold=(st, c, 1e-5, m1, r1), target_rows=True)
    torch.cuda.synchronize()
    assert abs(parts0.sum().item() - parts1.sum().item()) <= 1e-5 * abs(parts0.sum().item()) + 1e-7
    assert (g0.float() - g1.float()).abs().max().item() <= 1e-6
    # (row statistics summed in a different fixed order: last-bit differences)
    assert torch.allclose(m0, m1, rtol=1e-5, atol=1e-6) and torch.allclose(r0, r1, rtol=1e-5)
    assert g1.view(B, NP + 1, F)[:, 0].abs().max().item() == 0.0  # cls rows: zero gradient


@pytest.mark.gpu
@pytest.mark.parametrize("gauss", [False, True])
def test_fused_batch_target_rows(gauss):
    """The fused batch draw's patch-row target == image_to_rows of its image target."""
    from ddim_cold_amd.data.synthetic import SITE_DATA, SITE_NOISE, synthetic_pool
    from ddim_cold_amd.models.program import SITE_EMBED
    torch.manual_seed(0)
    model = build_model("vit_tiny").to(DEV).train()
    B, D, p = 8, model.embed_dim, 8
    N = model.patch_embed.num_patches + 1
    pool = synthetic_pool(32, seed=2, device=DEV)
    rng = torch.tensor([11, 5], dtype=torch.int64, device=DEV)
    pe_w = model.patch_embed.proj.weight.detach().reshape(D, -1).to(torch.bfloat16).contiguous()
    args = (pe_w, model.patch_embed.proj.bias.detach(), model.cls_token.detach(), model.pos_embed.detach(),
            model.time_embed.weight.detach(), rng, SITE_EMBED, 0.1, p)
    outs = []
    for rows in (False, True):
        xt, tg = torch.empty(B, 3, 64, 64, device=DEV), torch.empty(B, 3, 64, 64, device=DEV)
        t, idx = torch.empty(B, dtype=torch.int64, device=DEV), torch.empty(B, dtype=torch.int64, device=DEV)
        st = torch.empty(B * N, D // 32, 2, device=DEV)
        xb = torch.empty(B * N, D, dtype=torch.bfloat16, device=DEV)
        spec = (pool, SITE_DATA, 6, True, gauss, tg, idx, False) + ((2000, SITE_NOISE) if gauss else (0, 0))
        x, pt = ops.patch_embed_cold_fwd(spec, xt, t, *args, ln_st=st, xb_out=xb, target_rows=rows)
        outs.append((x, pt, tg, t))
    torch.cuda.synchronize()
    (x0, p0, g0, t0), (x1, p1, g1, t1) = outs
    assert torch.equal(x0, x1) and torch.equal(p0, p1) and torch.equal(t0, t1)
    assert torch.equal(ops.image_to_rows(g0, p).reshape(g1.shape), g1)
