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
