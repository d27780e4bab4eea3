"""Every GEMM tile configuration against the fp32 references, in process
(``ops.gemm_tile`` forces the tile of every launch inside it):

  0 = 32x64, 1 = 64x64, 2 = 128x64, 3 = 128x128   (4 waves)
  4 = 256x128, 5 = 128x128                          (8 waves, 512-thread workgroups;
                                                     the automatic choice for M >= 16,384)

Shapes include the vit_small_200 training rows (M = 32 * 626 = 20,032, not a
multiple of 256), ragged M / N, the K = 1,152 QKV input gradient, and the
LayerNorm-fold consumer and producer epilogues."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from ddim_cold_amd import ops
from ddim_cold_amd.ops import reference as ref

DEV = "cuda"
TILES = [0, 1, 2, 3, 4, 5]


@pytest.fixture(autouse=True)
def _native():
    from ddim_cold_amd.ops import _ext
    _ext.load(raise_on_error=True)
    torch.manual_seed(0)


def rng(seed=1234, step=5):
    return torch.tensor([seed, step], dtype=torch.int64, device=DEV)


def close(a, b, atol, rtol=0.0, name=""):
    a, b = a.float(), b.float()
    err = (a - b).abs()
    bad = (~(err <= atol + rtol * b.abs())).sum().item()  # NaN counts as a mismatch
    assert bad == 0, f"{name}: {bad} mismatches, max err {err.max().item():.3e}"


def bf(*shape, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).to(torch.bfloat16)


@pytest.mark.parametrize("tile", TILES)
@pytest.mark.parametrize("B,N,H,D", [(32, 626, 6, 384), (3, 17, 2, 128)])
def test_qkv_tiles(tile, B, N, H, D):
    a, w, b = bf(B * N, D), bf(3 * D, D, scale=0.05), torch.randn(3 * D, device=DEV)
    with ops.gemm_tile(tile):
        out = ops.qkv_fwd(a, w, b, B, N, H)
    close(out, ref.qkv_fwd(a, w, b, B, N, H), 2e-2, 1e-2, f"qkv tile {tile}")


@pytest.mark.parametrize("tile", TILES)
@pytest.mark.parametrize("M,N,pd,pdp", [(20032, 626, 0.1, 0.1), (4100, 25, 0.0, 0.3)])
def test_residual_producer_tiles(tile, M, N, pd, pdp):
    K = Nout = 384
    a, w, b = bf(M, K), bf(Nout, K, scale=0.05), torch.randn(Nout, device=DEV)
    x = torch.randn(M, Nout, device=DEV)
    r = rng()
    st = torch.full((M, Nout // 32, 2), float("nan"), device=DEV)  # every slot must be written
    xb = torch.empty(M, Nout, dtype=torch.bfloat16, device=DEV)
    with ops.gemm_tile(tile):
        y = ops.linear_residual_fwd(a, w, b, x, N, r, 3, pd, 4, pdp, st_out=st, xb_out=xb)
    close(y, ref.linear_residual_fwd(a, w, b, x, N, r, 3, pd, 4, pdp), 1e-3, 1e-4, f"resid tile {tile}")
    close(xb, y.to(torch.bfloat16), 0, 0, "bf16 copy")
    close(st, ref.row_stats(y), 1e-3, 1e-4, "row statistics slots")


@pytest.mark.parametrize("tile", TILES)
def test_gelu_fold_tiles(tile):
    M, K, Hm = 20032, 384, 384
    x = torch.randn(M, K, device=DEV) * 2 + 0.5
    st = ref.row_stats(x)
    w = torch.randn(Hm, K, device=DEV) * 0.05
    g, be, b = torch.randn(K, device=DEV), torch.randn(K, device=DEV), torch.randn(Hm, device=DEV)
    wf = torch.empty(Hm, K, dtype=torch.bfloat16, device=DEV)
    c, bfv = torch.empty(Hm, device=DEV), torch.empty(Hm, device=DEV)
    ops.ln_fold_([w], [g], [be], [b], [wf], [c], [bfv])
    xb = x.to(torch.bfloat16)
    r = rng()
    mean, rstd = torch.empty(M, device=DEV), torch.empty(M, device=DEV)
    with ops.gemm_tile(tile):
        u, h = ops.linear_gelu_fwd(xb, wf, bfv, r, 9, 0.1, fold=(st, c, 1e-5, mean, rstd))
        y = ops.linear_fwd(xb, wf, bfv, True, fold=(st, c, 1e-5))
    ur, hr = ref.linear_gelu_fwd(xb, wf, bfv, r, 9, 0.1, st, c, 1e-5)
    close(u, ur, 2e-2, 1e-2, "u")
    close(h, hr, 2e-2, 1e-2, "h")
    close(mean, x.mean(-1), 1e-4, 1e-4, "mean")
    close(y, ref.linear_fwd(xb, wf, bfv, True, st, c, 1e-5), 2e-3, 1e-3, "linear fold f32")


@pytest.mark.parametrize("tile", TILES)
@pytest.mark.parametrize("M,Nout,K", [(20032, 1152, 384), (20032, 384, 384), (4100, 384, 1152), (300, 200, 48)])
def test_dgrad_tiles(tile, M, Nout, K):
    dy, w = bf(M, Nout), bf(Nout, K, scale=0.05)
    with ops.gemm_tile(tile):
        d32 = ops.linear_dgrad(dy, w, True)
        d16 = ops.linear_dgrad(dy, w, False)
    close(d32, ref.linear_dgrad(dy, w, True), 1e-3, 1e-2, f"dgrad f32 tile {tile}")
    close(d16, ref.linear_dgrad(dy, w, False), 2e-2, 1e-2, f"dgrad bf16 tile {tile}")


@pytest.mark.parametrize("tile", TILES)
def test_dgrad_gelu_tiles(tile):
    M, N, K = 20032, 384, 384
    dy, w, u = bf(M, N), bf(N, K, scale=0.05), bf(M, K)
    r = rng()
    with ops.gemm_tile(tile):
        du = ops.linear_dgrad_gelu(dy, w, u, r, 11, 0.1)
    close(du, ref.linear_dgrad_gelu(dy, w, u, r, 11, 0.1), 2e-2, 1e-2, f"dgelu tile {tile}")


@pytest.mark.parametrize("tile", TILES)
def test_patch_embed_tiles(tile):
    B, C, H, W, p, D, pd = 32, 3, 200, 200, 8, 384, 0.1
    N = (H // p) * (W // p) + 1
    img = torch.randn(B, C, H, W, device=DEV)
    t = torch.randint(0, 2000, (B,), device=DEV)
    w = bf(D, C * p * p, scale=0.05)
    b, cls, pos = torch.randn(D, device=DEV), torch.randn(D, device=DEV), torch.randn(N, D, device=DEV)
    temb = torch.randn(2000, D, device=DEV)
    r = rng()
    with ops.gemm_tile(tile):
        x, _ = ops.patch_embed_fwd(img, t, w, b, cls, pos, temb, r, 1, pd, p)
    xr, _ = ref.patch_embed_fwd(img, t, w, b, cls, pos, temb, r, 1, pd, p)
    close(x, xr, 1e-3, 1e-3, f"tokens tile {tile}")


def test_tile_override_restores_and_rejects():
    with ops.gemm_tile(4):
        with ops.gemm_tile(2):
            pass
        assert int(torch.ops.ddim_cold.gemm_tile_override(4)) == 4
    assert int(torch.ops.ddim_cold.gemm_tile_override(-1)) == -1
    with pytest.raises(RuntimeError):
        torch.ops.ddim_cold.gemm_tile_override(9)
    # the head epilogues reduce over 4 waves: an 8-wave override fails loudly
    a, w, b = bf(34, 64), bf(48, 64, scale=0.05), torch.randn(48, device=DEV)  # B=2, 17 tokens
    with ops.gemm_tile(4), pytest.raises(RuntimeError):
        ops.head_fwd(a, w, b, 2, 3, 16, 16, 4)
        torch.cuda.synchronize()
