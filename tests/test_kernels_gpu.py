"""Numerics of every hand-written HIP kernel vs the plain-PyTorch fp32 reference.

Each test runs the op through ``torch.ops.ddim_cold`` (gfx950 kernel) and through
:mod:`ddim_cold_amd.ops.reference` on the same GPU inputs (the reference is
ordinary PyTorch fp32 math with the same bf16 rounding points and the same
counter-hash dropout masks), then compares.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

from ddim_cold_amd import ops
from ddim_cold_amd.ops import reference as ref

DEV = "cuda"


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
    tol = atol + rtol * b.abs()
    bad = (~(err <= tol)).sum().item()  # NaN counts as a mismatch
    assert bad == 0, f"{name}: {bad} mismatches, max err {err.max().item():.3e}"


def bf(*shape, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).to(torch.bfloat16)


# ------------------------------------------------------------------ LayerNorm
@pytest.mark.parametrize("M,D", [(2080, 384), (8224, 256), (37, 128), (100, 768)])
def test_layernorm_fwd(M, D):
    x = torch.randn(M, D, device=DEV) * 3 + 1
    g = torch.randn(D, device=DEV)
    b = torch.randn(D, device=DEV)
    y, mu, rs = ops.layernorm_fwd(x, g, b, 1e-5)
    yr, mur, rsr = ref.layernorm_fwd(x, g, b, 1e-5)
    close(mu, mur, 1e-5, 1e-5, "mean")
    close(rs, rsr, 1e-5, 1e-4, "rstd")
    close(y, yr, 2e-2, 1e-2, "y")


@pytest.mark.parametrize("emit,p", [(True, 0.1), (False, 0.0), (True, 0.0)])
def test_layernorm_bwd(emit, p):
    M, D, N = 2080, 384, 65
    x = torch.randn(M, D, device=DEV)
    g = torch.randn(D, device=DEV)
    b = torch.randn(D, device=DEV)
    _, mu, rs = ref.layernorm_fwd(x, g, b)
    dy = torch.randn(M, D, device=DEV)
    gres = torch.randn(M, D, device=DEV)
    dg1, db1 = torch.zeros(D, device=DEV), torch.zeros(D, device=DEV)
    dg2, db2 = torch.zeros(D, device=DEV), torch.zeros(D, device=DEV)
    r = rng()
    go, gy = ops.layernorm_bwd(dy, x, mu, rs, g, gres, dg1, db1, N, r, 7, p, 8, 0.2 if p else 0.0, emit)
    gor, gyr = ref.layernorm_bwd(dy, x, mu, rs, g, gres, dg2, db2, N, r, 7, p, 8, 0.2 if p else 0.0, emit)
    close(go, gor, 1e-4, 1e-4, "g_out")
    close(dg1, dg2, 1e-2, 1e-4, "dgamma")
    close(db1, db2, 1e-2, 1e-4, "dbeta")
    if emit:
        close(gy, gyr, 1e-2, 1e-2, "gy")
    else:
        assert gy is None


@pytest.mark.parametrize("M,D,N", [(2080, 384, 65), (20032, 384, 626), (8224, 256, 257), (40, 128, 5)])
def test_layernorm_bwd_workspace_deterministic(M, D, N):
    """dgamma||dbeta through the slot workspace (one slot per workgroup, workgroup-strided
    rows past 512 workgroups, slots summed in order by replica_reduce_): == the fp32
    oracle and BIT-identical over repeated launches (no fp32 atomics).  gp_out (the
    last LayerNorm of a backward) == the embedding backward's patch-row gradient."""
    x = torch.randn(M, D, device=DEV)
    g, b = torch.randn(D, device=DEV), torch.randn(D, device=DEV)
    _, mu, rs = ref.layernorm_fwd(x, g, b)
    dy, gres = torch.randn(M, D, device=DEV), torch.randn(M, D, device=DEV)
    r = rng()
    R = ops.ln_ws_rows(M)
    assert R == max(1, min(-(-M // 8), 512))
    ws = torch.zeros(1, R, 2 * D, device=DEV)
    outs = []
    for _ in range(3):
        z = torch.zeros(D, device=DEV)
        gp = torch.empty(M // N * (N - 1), D, dtype=torch.bfloat16, device=DEV)
        go, gy = ops.layernorm_bwd(dy, x, mu, rs, g, gres, z, z.clone(), N, r, 7, 0.1, 8, 0.2, True, ws[0],
                                   gp_out=gp, site_emb=1, p_emb=0.1)
        dst = torch.zeros(2 * D, device=DEV)
        ops.replica_reduce_(ws, torch.tensor([dst.data_ptr()], dtype=torch.int64, device=DEV), 2 * D, R)
        torch.cuda.synchronize()
        outs.append((go, gy, dst, gp))
    for go, gy, dst, gp in outs[1:]:
        assert torch.equal(go, outs[0][0]) and torch.equal(gy, outs[0][1]) and torch.equal(gp, outs[0][3])
        assert torch.equal(dst, outs[0][2]), "dgamma||dbeta differ between identical launches"
    dg2, db2 = torch.zeros(D, device=DEV), torch.zeros(D, device=DEV)
    gor, _ = ref.layernorm_bwd(dy, x, mu, rs, g, gres, dg2, db2, N, r, 7, 0.1, 8, 0.2, True)
    close(outs[0][2][:D], dg2, 2e-3 * dg2.abs().max().item(), 1e-4, "dgamma")
    close(outs[0][2][D:], db2, 2e-3 * db2.abs().max().item(), 1e-4, "dbeta")
    close(outs[0][0], gor, 1e-4, 1e-4, "g_out")
    gpr = ref.embed_patch_grad(outs[0][0].view(-1, N, D), r, 1, 0.1)
    close(outs[0][3], gpr, 2e-2, 1e-2, "patch-row gradient")
    assert torch.equal(outs[0][3] == 0, gpr == 0), "embedding dropout masks differ"


# ------------------------------------------------------------------ GEMMs
# (32, 626, 6, 384): vit_small_200's M = 20,032 -> the 256x192 2-stage tiles (gemm.hip Big192);
# (27, 626, 6, 384): M = 16,902, a partial last row tile of those
@pytest.mark.parametrize("B,N,H,D", [(32, 65, 12, 384), (4, 257, 4, 256), (3, 17, 2, 64 * 2), (32, 626, 6, 384),
                                     (27, 626, 6, 384)])
def test_qkv_fwd(B, N, H, D):
    a = bf(B * N, D)
    w = bf(3 * D, D, scale=0.05)
    b = torch.randn(3 * D, device=DEV)
    out = ops.qkv_fwd(a, w, b, B, N, H)
    outr = ref.qkv_fwd(a, w, b, B, N, H)
    assert out.shape == (3, B, H, N, D // H)
    close(out, outr, 2e-2, 1e-2, "qkv")


@pytest.mark.parametrize("M,K,Nout,pd,pdp", [(2080, 384, 384, 0.1, 0.1), (2080, 384, 384, 0.0, 0.0),
                                              (8224, 256, 256, 0.1, 0.0), (100, 48, 40, 0.0, 0.3)])
def test_linear_residual(M, K, Nout, pd, pdp):
    N = 65 if M % 65 == 0 else (257 if M % 257 == 0 else M // 4 if M % 4 == 0 else M)
    a = bf(M, K)
    w = bf(Nout, K, scale=0.05)
    b = torch.randn(Nout, device=DEV)
    x = torch.randn(M, Nout, device=DEV)
    r = rng()
    y = ops.linear_residual_fwd(a, w, b, x, N, r, 3, pd, 4, pdp)
    yr = ref.linear_residual_fwd(a, w, b, x, N, r, 3, pd, 4, pdp)
    close(y, yr, 1e-3, 1e-4, "resid")


def test_gemm_asymmetric_identity():
    """A = I with an asymmetric B catches a transposed C write (guide §3)."""
    K = 64
    a = torch.eye(K, device=DEV).to(torch.bfloat16)
    w = (torch.arange(K * K, device=DEV).float().view(K, K) % 97 / 97.0).to(torch.bfloat16)
    x = torch.zeros(K, K, device=DEV)
    y = ops.linear_residual_fwd(a, w, torch.zeros(K, device=DEV), x, K, rng(), 0, 0.0, 0, 0.0)
    close(y, w.float().t(), 1e-6, 0, "identity")


def test_linear_gelu():
    M, K, Hm = 2080, 384, 384
    a, w, b = bf(M, K), bf(Hm, K, scale=0.05), torch.randn(Hm, device=DEV)
    r = rng()
    u, h = ops.linear_gelu_fwd(a, w, b, r, 9, 0.1)
    ur, hr = ref.linear_gelu_fwd(a, w, b, r, 9, 0.1)
    close(u, ur, 2e-2, 1e-2, "u")
    close(h, hr, 2e-2, 1e-2, "h")


@pytest.mark.parametrize("B,C,H,W,p,D", [(4, 3, 64, 64, 8, 384), (2, 3, 64, 64, 4, 256), (2, 3, 200, 200, 8, 384)])
def test_head_fwd(B, C, H, W, p, D):
    N = (H // p) * (W // p) + 1
    a = bf(B * N, D)
    w = bf(C * p * p, D, scale=0.05)
    b = torch.randn(C * p * p, device=DEV)
    img = ops.head_fwd(a, w, b, B, C, H, W, p)
    imgr = ref.head_fwd(a, w, b, B, C, H, W, p)
    close(img, imgr, 1e-3, 1e-3, "head")


@pytest.mark.parametrize("mode", [1, 2])
def test_head_step_fused_sampler_update(mode):
    """Head GEMM with the DDIM update (mode 1) / clamp (mode 2) in its epilogue."""
    from ddim_cold_amd.diffusion.schedule import ddim_coefficients
    B, C, H, W, p, D = 4, 3, 64, 64, 8, 384
    N = (H // p) * (W // p) + 1
    a = bf(B * N, D)
    w = bf(C * p * p, D, scale=0.05)
    b = torch.randn(C * p * p, device=DEV)
    x = torch.randn(B, C, H, W, device=DEV)
    coef = torch.tensor(ddim_coefficients(2000, 999, 20), device=DEV)
    x0 = torch.empty_like(x)
    xk = x.clone()
    ops.head_step_(a, w, b, xk, x0 if mode == 1 else None, coef if mode == 1 else None, p, mode)
    raw = ref.head_fwd(a, w, b, B, C, H, W, p)
    if mode == 2:
        close(xk, raw.clamp(-1, 1), 1e-3, 1e-3, "clamp")
    else:
        xn, x0r = ref.ddim_step(x, raw, coef.tolist())
        close(x0, x0r, 1e-3, 1e-3, "x0")
        close(xk, xn, 2e-3, 1e-3, "x_next")


def test_head_step_per_sample_coefficients():
    """Mode 4 (img2img): one coefficient row per sample; the identity row {0,1,0,1}
    leaves a not-yet-started sample's x_t bit-identical; the patch rows handed to
    the next step match the new x."""
    from ddim_cold_amd.diffusion.schedule import ddim_coefficients
    B, C, H, W, p, D = 5, 3, 64, 64, 8, 384
    N = (H // p) * (W // p) + 1
    a = bf(B * N, D)
    w = bf(C * p * p, D, scale=0.05)
    b = torch.randn(C * p * p, device=DEV)
    x = torch.randn(B, C, H, W, device=DEV)
    rows = [ddim_coefficients(2000, t, 10) for t in (1999, 1599, 999)] + [(0.0, 1.0, 0.0, 1.0)] * 2
    coef = torch.tensor(rows, device=DEV)
    x0 = torch.empty_like(x)
    xk = x.clone()
    pout = torch.empty(B * (N - 1), C * p * p, dtype=torch.bfloat16, device=DEV)
    ops.head_step_(a, w, b, xk, x0, coef, p, 4, patches_out=pout)
    raw = ref.head_fwd(a, w, b, B, C, H, W, p)
    for i in range(B):
        xn, x0r = ref.ddim_step(x[i:i + 1], raw[i:i + 1], rows[i])
        close(xk[i:i + 1], xn, 2e-3, 1e-3, f"x_next[{i}]")
        close(x0[i:i + 1], x0r, 1e-3, 1e-3, f"x0[{i}]")
    assert torch.equal(xk[3:], x[3:])  # identity rows: exactly unchanged
    close(pout.float(), ref.patchify_bf16(xk, p).reshape(B * (N - 1), -1).float(), 0, 0, "patch rows")


@pytest.mark.parametrize("B,C,H,W,p,D,pd", [(4, 3, 64, 64, 8, 384, 0.1), (2, 3, 64, 64, 4, 256, 0.0),
                                            (2, 3, 64, 64, 16, 128, 0.1)])  # p=16: the generic segment path
def test_patch_embed(B, C, H, W, p, D, pd):
    N = (H // p) * (W // p) + 1
    img = torch.randn(B, C, H, W, device=DEV)
    t = torch.randint(0, 2000, (B,), device=DEV)
    w = bf(D, C * p * p, scale=0.05)
    b, cls, pos = torch.randn(D, device=DEV), torch.randn(D, device=DEV), torch.randn(N, D, device=DEV)
    temb = torch.randn(2000, D, device=DEV)
    r = rng()
    x, pt = ops.patch_embed_fwd(img, t, w, b, cls, pos, temb, r, 1, pd, p)
    xr, ptr = ref.patch_embed_fwd(img, t, w, b, cls, pos, temb, r, 1, pd, p)
    close(pt, ptr, 0, 0, "patches")
    close(x, xr, 1e-3, 1e-3, "tokens")


@pytest.mark.parametrize("M,Nout,K", [(2080, 384, 384), (2080, 1152, 384), (2080, 192, 384), (8224, 256, 256),
                                      (100, 48, 40)])
def test_dgrad(M, Nout, K):
    dy = bf(M, Nout)
    w = bf(Nout, K, scale=0.05)
    for fp32 in (True, False):
        dx = ops.linear_dgrad(dy, w, fp32)
        dxr = ref.linear_dgrad(dy, w, fp32)
        close(dx, dxr, 2e-2 if not fp32 else 1e-3, 1e-2, f"dgrad fp32={fp32}")


@pytest.mark.parametrize("M,Nout,K,splits", [(2080, 1152, 384, 2), (2080, 1152, 384, 3), (300, 768, 256, 4),
                                             (100, 200, 48, 2)])
def test_dgrad_ksplit(M, Nout, K, splits):
    """K-split dgrad: per-slice partial products (no atomics) and the LayerNorm
    backward summing them on load."""
    dy = bf(M, Nout)
    w = bf(Nout, K, scale=0.05)
    dx = ops.linear_dgrad(dy, w, True, splits)
    dxr = ref.linear_dgrad(dy, w, True, splits)
    assert dx.shape == (splits, M, K)
    close(dx, dxr, 1e-3, 1e-2, "dgrad slices")
    close(dx.sum(0), ref.linear_dgrad(dy, w, True), 1e-3, 1e-2, "dgrad sum")
    if K % 128 == 0:
        x = torch.randn(M, K, device=DEV)
        g, b = torch.randn(K, device=DEV), torch.randn(K, device=DEV)
        _, mu, rs = ref.layernorm_fwd(x, g, b)
        dg1, db1, dg2, db2 = (torch.zeros(K, device=DEV) for _ in range(4))
        go, _ = ops.layernorm_bwd(dx, x, mu, rs, g, None, dg1, db1, M, rng(), 0, 0.0, 0, 0.0, False)
        gor, _ = ref.layernorm_bwd(dx.sum(0), x, mu, rs, g, None, dg2, db2, M, rng(), 0, 0.0, 0, 0.0, False)
        close(go, gor, 1e-4, 1e-4, "ln g_out (summed partials)")
        close(dg1, dg2, 1e-2, 1e-4, "ln dgamma (summed partials)")


@pytest.mark.parametrize("M,N,K", [(2080, 384, 384), (20032, 384, 384), (300, 256, 128)])
def test_dgrad_gelu(M, N, K):
    """dU = (dY W) * gelu'(u) with dropout; also from the transposed weight W^T (the
    k-contiguous operand path the long-sequence engine uses): same values, same masks."""
    dy, w, u = bf(M, N), bf(N, K, scale=0.05), bf(M, K)
    r = rng()
    du = ops.linear_dgrad_gelu(dy, w, u, r, 11, 0.1)
    dur = ref.linear_dgrad_gelu(dy, w, u, r, 11, 0.1)
    close(du, dur, 2e-2, 1e-2, "dgelu")
    dut = ops.linear_dgrad_gelu(dy, w, u, r, 11, 0.1, wt=w.t().contiguous())
    close(dut, dur, 2e-2, 1e-2, "dgelu (W^T)")
    assert torch.equal(dut == 0, dur == 0), "dropout masks differ"


@pytest.mark.parametrize("M,Nout,K", [(2080, 384, 384), (2080, 1152, 384), (2080, 192, 384), (8224, 256, 256),
                                      (2048, 384, 192), (100, 48, 40)])
def test_wgrad(M, Nout, K):
    dy, x = bf(M, Nout), bf(M, K)
    dw0 = torch.randn(Nout, K, device=DEV)
    db0 = torch.randn(Nout, device=DEV)
    dw1, db1 = dw0.clone(), db0.clone()
    ops.linear_wgrad(dy, x, dw1, db1)
    dw2, db2 = dw0.clone(), db0.clone()
    ref.linear_wgrad(dy, x, dw2, db2)
    close(dw1, dw2, 2e-2, 1e-4, "dw")
    close(db1, db2, 2e-2, 1e-4, "db")


@pytest.mark.parametrize("M,N,K,f32,bias", [(2080, 1152, 384, False, True), (100, 192, 64, True, False),
                                            (4160, 384, 384, True, True)])
def test_linear_fwd(M, N, K, f32, bias):
    a, w = bf(M, K), bf(N, K, scale=0.05)
    b = torch.randn(N, device=DEV) if bias else None
    y = ops.linear_fwd(a, w, b, f32)
    yr = ref.linear_fwd(a, w, b, f32)
    close(y.float(), yr.float(), 3e-2, 2e-2, "y")


@pytest.mark.parametrize("n,big", [(1, False), (7, False), (30, False), (5, True), (36, True)])
def test_linear_wgrad_multi(n, big):
    """Every weight gradient of a step in one launch == per-problem reference (bias or not, odd shapes).
    ``big``: a reduction over >= 16,384 tokens (vit_small_200: 128 x 128 tiles, 8 waves); there
    the tiles past the last whole round of 256 run as K pieces summed by the last one
    (5 problems: 60 tiles in 4 pieces; 36: two launches with balanced tile counts, each
    with a split tail)."""
    shapes = [(1152, 384), (384, 384), (384, 384), (384, 384), (192, 384), (384, 192), (64, 96), (256, 128)]
    jobs, refs = [], []
    for i in range(n):
        nout, k = shapes[i % len(shapes)]
        m = (20032 if i % 2 else 16500) if big else (2080 if i % 3 else 300)
        dy, x = bf(m, nout), bf(m, k)
        dw0 = torch.randn(nout, k, device=DEV) * 0.1
        db0 = torch.randn(nout, device=DEV) if i % 2 == 0 else None
        jobs.append((dy, x, dw0.clone(), db0.clone() if db0 is not None else None))
        dw2, db2 = dw0.clone(), (db0.clone() if db0 is not None else None)
        ref.linear_wgrad(dy, x, dw2, db2)
        refs.append((dw2, db2))
    ops.linear_wgrad_multi(jobs)
    for (_, _, dw, db), (dw2, db2) in zip(jobs, refs):
        close(dw, dw2, 2e-2, 1e-4, "dw")
        if db is not None:
            close(db, db2, 2e-2, 1e-4, "db")


def test_linear_wgrad_multi_vit_tiny_tiles():
    """ViT-tiny's 1,548 64 x 64 weight-gradient tiles (two launches' worth of problems,
    balanced) at a short reduction (K = 520 tokens) == the reference."""
    shapes = [(1152, 384), (384, 384), (384, 384), (384, 384)] * 7 + [(192, 384), (384, 192)]
    jobs, refs = [], []
    for i, (n, k) in enumerate(shapes):
        m = 520
        dy, x = bf(m, n), bf(m, k)
        dw, db = torch.randn(n, k, device=DEV), (torch.randn(n, device=DEV) if i % 2 == 0 else None)
        dw2, db2 = dw.clone(), (db.clone() if db is not None else None)
        ref.linear_wgrad(dy, x, dw2, db2)
        jobs.append((dy, x, dw, db))
        refs.append((dw2, db2))
    ops.linear_wgrad_multi(jobs)
    for (_, _, dw, db), (dw2, db2) in zip(jobs, refs):
        close(dw, dw2, 2e-2, 1e-4, "dw")
        if db is not None:
            close(db, db2, 2e-2, 1e-4, "db")


def test_linear_wgrad_multi_split_tail_deterministic():
    """vit_small_200's weight gradients (24 problems of a 6-block half: 324 tiles = one whole
    round + 68 tiles in 3 K pieces): bit-identical over repeated launches (the pieces are
    summed in piece order by whichever finishes last) and == the reference."""
    shapes = [(1152, 384), (384, 384), (384, 384), (384, 384)] * 6
    data = [(bf(20032, n), bf(20032, k)) for n, k in shapes]
    outs = []
    for _ in range(3):
        jobs = [(dy, x, torch.zeros(dy.shape[1], x.shape[1], device=DEV), torch.zeros(dy.shape[1], device=DEV))
                for dy, x in data]
        ops.linear_wgrad_multi(jobs, store=True)
        torch.cuda.synchronize()
        outs.append(jobs)
    for jobs in outs[1:]:
        for (_, _, dw, db), (_, _, dw0, db0) in zip(jobs, outs[0]):
            assert torch.equal(dw, dw0) and torch.equal(db, db0), "split-tail weight gradients differ between launches"
    for (dy, x, dw, db) in outs[0][-4:]:  # the last block's problems hold the split tiles
        dw2, db2 = torch.zeros_like(dw), torch.zeros_like(db)
        ref.linear_wgrad(dy, x, dw2, db2)
        close(dw, dw2, 2e-2, 1e-4, "dw")
        close(db, db2, 2e-2, 1e-4, "db")


@pytest.mark.parametrize("store", [False, True])
@pytest.mark.parametrize("lazy", [None, (64, 64 + 4 * 1000)])
@pytest.mark.parametrize("big", [False, True])
def test_linear_wgrad_multi_sqnorm_partials(store, lazy, big):
    """Grad-norm partials from the weight-gradient launch (engine FUSE_SQNORM): targets
    are views of one arena with gaps the tail workgroups cover (and a lazy range they
    skip); the partials sum to the arena's sum of squares, dW / db unchanged, unused
    slots zero, and the optimizer kernels accept the buffer."""
    shapes = [(1152, 384, True), (384, 384, True), (384, 1536, False), (192, 384, True), (64, 96, True)]
    if not big:  # 35 problems: two launches (<= 32 each), partials of the second after the first's
        shapes = shapes + [(64, 96, i % 2 == 0) for i in range(30)]
    sizes = [n * k + (n if b else 0) for n, k, b in shapes]
    lo0 = 64 + 4 * 1000 + 1000  # after the lazy range and a gap of "embedding" gradients
    arena = torch.zeros(lo0 + sum(sizes) + len(shapes) * 777 + 13, device=DEV)
    arena[:lo0].normal_()
    if lazy is not None:
        arena[lazy[0]:lazy[1]] = 0  # a lazy range has a zero gradient by construction
    off = lo0
    jobs, refs = [], []
    for i, (nout, k, hb) in enumerate(shapes):
        m = (20032 if i % 2 else 16400) if big else (2080 if i % 2 else 300)
        dy, x = bf(m, nout), bf(m, k)
        dw = arena[off:off + nout * k].view(nout, k)
        off += nout * k
        db = None
        if hb:
            db = arena[off:off + nout]
            off += nout
        if not store:
            dw.normal_()
            if db is not None:
                db.normal_()
        gap = 777 if i < 5 else 0  # gaps no tile writes (<= 16 ranges)
        arena[off:off + gap].normal_()
        off += gap
        dw2, db2 = dw.clone(), (db.clone() if db is not None else None)
        if store:
            dw2.zero_()
            if db2 is not None:
                db2.zero_()
        ref.linear_wgrad(dy, x, dw2, db2)
        refs.append((dw2, db2))
        jobs.append((dy, x, dw, db))
    parts = torch.full((ops.sq_parts_size(3000),), float("nan"), device=DEV)
    ops.linear_wgrad_multi(jobs, store=store, sq=(parts, arena, lazy))
    for (_, _, dw, db), (dw2, db2) in zip(jobs, refs):
        close(dw, dw2, 2e-2, 1e-4, "dw")
        if db is not None:
            close(db, db2, 2e-2, 1e-4, "db")
    assert torch.isfinite(parts).all(), "every partial slot is written"
    expect = arena.double().pow(2).sum().item()
    got = parts.double().sum().item()
    assert abs(got - expect) <= 1e-5 * expect, (got, expect)
    # the sqnorm kernel writes the same quantity into the same layout
    parts2 = torch.empty_like(parts)
    ops.sqnorm(arena, parts2, 1.0, lazy=lazy)
    assert abs(parts2.double().sum().item() - expect) <= 1e-5 * expect
    with pytest.raises(RuntimeError, match="grad-norm partials"):
        ops.linear_wgrad_multi(jobs, sq=(torch.zeros(256, device=DEV), arena, lazy))
    with pytest.raises(RuntimeError, match="outside the arena"):
        ops.linear_wgrad_multi(jobs, sq=(parts, arena[:lo0], None))


# ------------------------------------------------------------------ attention
@pytest.mark.parametrize("B,H,N,hd,p", [(4, 12, 65, 32, 0.0), (4, 12, 65, 32, 0.1), (2, 4, 257, 64, 0.1),
                                        (1, 2, 17, 32, 0.0), (1, 6, 626, 64, 0.0), (2, 3, 130, 64, 0.2),
                                        # short-sequence path (N <= 128): every padded size, both head dims
                                        (2, 3, 100, 64, 0.1), (3, 5, 128, 32, 0.1), (2, 2, 64, 64, 0.0),
                                        (2, 4, 32, 32, 0.1), (2, 4, 33, 64, 0.0), (8, 4, 97, 32, 0.0),
                                        # resident-KV forward (128 < N <= 320, B*H >= 192)
                                        (48, 4, 257, 64, 0.1), (16, 12, 200, 32, 0.0),
                                        # flash v2 (N >= 384)
                                        (1, 2, 400, 32, 0.1), (2, 3, 513, 64, 0.0)])
def test_attention_fwd_bwd(B, H, N, hd, p):
    qkv = bf(3, B, H, N, hd)
    r = rng()
    scale = hd ** -0.5
    o, lse = ops.attn_fwd(qkv, scale, r, 5, p)
    or_, lser = ref.attn_fwd(qkv, scale, r, 5, p)
    close(lse, lser, 1e-3, 1e-4, "lse")
    close(o, or_, 2e-2, 2e-2, "o")
    do = bf(B, N, H * hd)
    dq = ops.attn_bwd(do, qkv, o, lse, scale, r, 5, p)
    dqr = ref.attn_bwd(do, qkv, o, lse, scale, r, 5, p)
    assert dq.shape == (B * N, 3 * H * hd)
    close(dq, dqr, 3e-2, 3e-2, "dqkv")
    # keep flags stored by the forward == masks re-hashed in the backward, bit for bit
    keep = ops.attn_keep_buffer(qkv, p)
    if keep is not None:
        o2, lse2 = ops.attn_fwd(qkv, scale, r, 5, p, keep_out=keep)
        assert torch.equal(o2, o) and torch.equal(lse2, lse)
        assert torch.equal(ops.attn_bwd(do, qkv, o, lse, scale, r, 5, p, keep=keep), dq)


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_attention_n2501(p):
    """The 200x200 / p=4 sequence length (2,501 tokens, 40 key tiles, ragged tail) the
    long-sequence kernels are benchmarked at: forward, backward, stored keep words."""
    B, H, N, hd = 2, 2, 2501, 64
    qkv = bf(3, B, H, N, hd)
    r = rng()
    scale = hd ** -0.5
    keep = ops.attn_keep_buffer(qkv, p)
    assert (keep is not None) == (p > 0) and (keep is None or keep.numel() == B * H * N * 40 * 2)
    o, lse = ops.attn_fwd(qkv, scale, r, 5, p, keep_out=keep)
    or_, lser = ref.attn_fwd(qkv, scale, r, 5, p)
    close(lse, lser, 1e-3, 1e-4, "lse")
    close(o, or_, 2e-2, 2e-2, "o")
    do = bf(B, N, H * hd)
    dq = ops.attn_bwd(do, qkv, o, lse, scale, r, 5, p, keep=keep)
    close(dq, ref.attn_bwd(do, qkv, o, lse, scale, r, 5, p), 3e-2, 3e-2, "dqkv")
    if keep is not None:  # stored words == re-hashed masks, bit for bit
        assert torch.equal(ops.attn_bwd(do, qkv, o, lse, scale, r, 5, p), dq)


def test_attention_mask_index_beyond_2p31():
    """Dropout mask indices are 32-bit counters (hoisted pair-hash math): at B*H = 400,
    N = 2,501 they pass 2^31 (signed overflow would show here).  The last head (mask
    indices ~2.5e9) against the reference's mask for that slice; stored keep words vs
    re-hashing over the whole batch."""
    B, H, N, hd, p = 1, 400, 2501, 64, 0.1
    assert (B * H - 1) * N * ((N + 3) // 4 * 4) > 2 ** 31
    qkv = bf(3, B, H, N, hd)
    r = rng()
    scale = hd ** -0.5
    keep = ops.attn_keep_buffer(qkv, p)
    o, lse = ops.attn_fwd(qkv, scale, r, 5, p, keep_out=keep)
    last = qkv[:, :, H - 1:].contiguous()
    or_, lser = ref.attn_fwd(last, scale, r, 5, p, bh0=H - 1)
    D = H * hd
    close(lse[:, H - 1:], lser, 1e-3, 1e-4, "lse (last head)")
    close(o[:, :, D - hd:], or_, 2e-2, 2e-2, "o (last head)")
    do = bf(B, N, D)
    dq = ops.attn_bwd(do, qkv, o, lse, scale, r, 5, p, keep=keep)
    dqr = ref.attn_bwd(do[:, :, D - hd:].contiguous(), last, o[:, :, D - hd:].contiguous(), lse[:, H - 1:].contiguous(),
                       scale, r, 5, p, bh0=H - 1)
    dqv = dq.view(B * N, 3, D)[:, :, D - hd:].reshape(B * N, 3 * hd)
    close(dqv, dqr, 3e-2, 3e-2, "dqkv (last head)")
    assert torch.equal(ops.attn_bwd(do, qkv, o, lse, scale, r, 5, p), dq)


def test_attention_mask_index_guard():
    """More than 2^32 mask elements: refused before launch (dropout on); fine without."""
    B, H, N, hd = 1, 700, 2501, 32
    assert B * H * N * ((N + 3) // 4 * 4) >= 2 ** 32
    qkv = torch.zeros(3, B, H, N, hd, dtype=torch.bfloat16, device=DEV)
    with pytest.raises(RuntimeError, match="2\\^32"):
        ops.attn_fwd(qkv, hd ** -0.5, rng(), 5, 0.1)


def test_attention_spike_rescale():
    """Force a running-max jump at the second KV tile (online-softmax rescale branch)."""
    B, H, N, hd = 1, 1, 130, 32
    qkv = bf(3, B, H, N, hd, scale=0.5)
    qkv[1, 0, 0, 100] = 8.0   # one key far to the right with a large dot product
    qkv[0, 0, 0, :] = 8.0
    r = rng()
    o, lse = ops.attn_fwd(qkv, hd ** -0.5, r, 5, 0.0)
    or_, lser = ref.attn_fwd(qkv, hd ** -0.5, r, 5, 0.0)
    close(lse, lser, 1e-3, 1e-4, "lse")
    close(o, or_, 2e-2, 2e-2, "o")


@pytest.mark.parametrize("B,H,N,hd,p", [(1, 2, 700, 64, 0.0), (1, 2, 700, 64, 0.1), (2, 1, 1030, 32, 0.0),
                                        (48, 4, 300, 64, 0.0), (48, 4, 300, 64, 0.1)])
def test_attention_lazy_max_ramp(B, H, N, hd, p):
    """Flash / resident forwards keep a lazy running max (it moves only when a tile's
    max exceeds it by 2^8).  Scores that ramp up along the keys, at a different slope
    per query, make that rescale branch fire at different tiles for different lanes
    of one wave (and not at all for flat rows): every case against the reference."""
    g = torch.Generator(device=DEV).manual_seed(3)
    u = torch.randn(hd, device=DEV, generator=g)
    u = u / u.norm()
    a = torch.linspace(0.0, 40.0, N, device=DEV)[torch.randperm(N, device=DEV, generator=g)]  # per-query slope
    b = torch.linspace(0.0, 8.0, N, device=DEV)                                            # key ramp
    qkv = torch.empty(3, B, H, N, hd, device=DEV)
    qkv[0] = a[:, None] * u + 0.05 * torch.randn(B, H, N, hd, device=DEV, generator=g)
    qkv[1] = b[:, None] * u + 0.05 * torch.randn(B, H, N, hd, device=DEV, generator=g)
    qkv[2] = torch.randn(B, H, N, hd, device=DEV, generator=g)
    qkv = qkv.to(torch.bfloat16)
    r = rng()
    scale = hd ** -0.5
    o, lse = ops.attn_fwd(qkv, scale, r, 5, p)
    or_, lser = ref.attn_fwd(qkv, scale, r, 5, p)
    close(lse, lser, 1e-3, 1e-4, "lse")
    close(o, or_, 2e-2, 2e-2, "o")
    do = bf(B, N, H * hd)
    close(ops.attn_bwd(do, qkv, o, lse, scale, r, 5, p), ref.attn_bwd(do, qkv, o, lse, scale, r, 5, p),
          3e-2, 3e-2, "dqkv")


# ------------------------------------------------------------------ embedding / loss
@pytest.mark.parametrize("B,N,D", [(32, 65, 384), (4, 626, 384), (3, 257, 256)])  # 2, 10 and 5 token chunks
def test_embed_bwd(B, N, D):
    g = torch.randn(B, N, D, device=DEV)
    t = torch.tensor(([3, 3, 7] + list(range(100, 129)))[:B], device=DEV)
    r = rng()
    outs = []
    for fn in (ops.embed_bwd, ref.embed_bwd):
        dcls, dpos, dtemb = torch.zeros(D, device=DEV), torch.zeros(N, D, device=DEV), torch.zeros(2000, D, device=DEV)
        gp = fn(g, t, r, 1, 0.1, dcls, dpos, dtemb)
        outs.append((gp, dcls, dpos, dtemb))
    for a, b, n in zip(outs[0], outs[1], ["gpatch", "dcls", "dpos", "dtemb"]):
        close(a, b, 2e-2 if n == "gpatch" else 1e-3, 1e-3, n)


@pytest.mark.parametrize("B,N,D,tset", [(32, 65, 384, "cold"), (32, 626, 384, "cold"), (32, 65, 384, "gauss"),
                                        (300, 17, 128, "cold")])
def test_embed_bwd_time_embedding_deterministic(B, N, D, tset):
    """The time-embedding gradient is summed per distinct timestep in sample order (no
    fp32 atomics): bit-identical across launches, == the fp32 oracle; more than 256
    samples take extra part-B passes (300 samples)."""
    g = torch.randn(B, N, D, device=DEV)
    gen = torch.Generator().manual_seed(3)
    t = (torch.randint(1, 7, (B,), generator=gen) if tset == "cold" else torch.randint(0, 2000, (B,), generator=gen))
    t = t.to(DEV)
    r = rng()
    res = []
    for _ in range(3):
        dcls, dpos, dtemb = torch.zeros(D, device=DEV), torch.zeros(N, D, device=DEV), torch.zeros(2000, D, device=DEV)
        ops.embed_bwd(g, t, r, 1, 0.1, dcls, dpos, dtemb)
        torch.cuda.synchronize()
        res.append((dcls, dpos, dtemb))
    for o in res[1:]:
        assert all(torch.equal(a, b) for a, b in zip(o, res[0]))
    dcls, dpos, dtemb = torch.zeros(D, device=DEV), torch.zeros(N, D, device=DEV), torch.zeros(2000, D, device=DEV)
    ref.embed_bwd(g, t, r, 1, 0.1, dcls, dpos, dtemb)
    close(res[0][2], dtemb, 1e-3 * dtemb.abs().max().item(), 1e-3, "dtemb")
    close(res[0][1], dpos, 1e-3 * dpos.abs().max().item(), 1e-3, "dpos")
    untouched = torch.ones(2000, dtype=torch.bool, device=DEV)
    untouched[t] = False
    assert not res[0][2][untouched].any()


@pytest.mark.parametrize("p", [8, 4])
def test_smooth_l1(p):
    B, C, H, W = 8, 3, 64, 64
    N = (H // p) * (W // p) + 1
    pred = torch.randn(B, C, H, W, device=DEV) * 1.5
    tgt = torch.randn(B, C, H, W, device=DEV)
    loss, dt = ops.smooth_l1_fwd_bwd(pred, tgt, N, p, 1.0)
    lr_, dtr = ref.smooth_l1_fwd_bwd(pred, tgt, N, p, 1.0)
    torch.testing.assert_close(loss, lr_, rtol=1e-4, atol=1e-6)
    ref_loss = torch.nn.functional.smooth_l1_loss(pred, tgt)
    torch.testing.assert_close(loss[0], ref_loss, rtol=1e-4, atol=1e-6)
    close(dt, dtr, 1e-9, 1e-2, "dtok")
    dimg = torch.randn(B, C, H, W, device=DEV)
    close(ops.img_to_tokgrad(dimg, N, p), ref.img_to_tokgrad(dimg, N, p), 0, 1e-2, "tokgrad")


# ------------------------------------------------------------------ optimizer
def test_fused_adamw_matches_torch():
    torch.manual_seed(1)
    n = 100_003
    p0 = torch.randn(n, device=DEV)
    steps = 4
    # torch reference: AdamW(wd=0.05) + clip 1.0 + cosine LR (per-step)
    pt = p0.clone().requires_grad_(True)
    opt = torch.optim.AdamW([pt], lr=3e-3, weight_decay=0.05)
    sch = torch.optim.lr_scheduler.CosineAnnealingLR(opt, 10, 0.0)
    # fused
    p, g, m, v = p0.clone(), torch.zeros(n, device=DEV), torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    pb = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    sq = torch.zeros(ops.SQ_PARTS, device=DEV)
    step = torch.zeros(2, dtype=torch.int64, device=DEV)
    r = rng()
    hyper = torch.tensor([3e-3, 0.9, 0.999, 1e-8, 0.05, 1.0, 10.0, 0.0], device=DEV)
    for s in range(steps):
        grad = torch.randn(n, device=DEV) * (0.001 if s % 2 else 0.1)
        pt.grad = grad.clone()
        torch.nn.utils.clip_grad_norm_([pt], 1.0)
        opt.step()
        sch.step()
        g.copy_(grad)
        ops.sqnorm(g, sq, 1.0)
        ops.adamw_step(p, g, m, v, pb, sq, step, hyper, 1.0)
        ops.advance_counters(step, r, sq)
    torch.testing.assert_close(p, pt.detach(), rtol=1e-5, atol=1e-6)
    assert torch.all(g == 0)
    close(pb, p, 1e-2, 1e-2, "bf16 shadow")
    assert step.tolist() == [steps, steps]


def test_fused_adamw_lazy_range_matches_torch():
    """Rows with identically zero gradient (cold training's unused time_embed rows) are
    skipped by the kernels; their accumulated decay, applied once, gives torch's AdamW."""
    torch.manual_seed(2)
    n, lo, hi = 100_004, 20_480, 97_280
    p0 = torch.randn(n, device=DEV)
    pt = p0.clone().requires_grad_(True)
    opt = torch.optim.AdamW([pt], lr=3e-3, weight_decay=0.05)
    sch = torch.optim.lr_scheduler.CosineAnnealingLR(opt, 10, 0.0)
    p, g, m, v = p0.clone(), torch.zeros(n, device=DEV), torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    pb = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    sq = torch.zeros(ops.SQ_PARTS, device=DEV)
    step = torch.zeros(2, dtype=torch.int64, device=DEV)
    lazy_decay = torch.ones(1, device=DEV)
    hyper = torch.tensor([3e-3, 0.9, 0.999, 1e-8, 0.05, 1.0, 10.0, 0.0], device=DEV)
    for s in range(4):
        grad = torch.randn(n, device=DEV) * (0.001 if s % 2 else 0.1)
        grad[lo:hi] = 0
        pt.grad = grad.clone()
        torch.nn.utils.clip_grad_norm_([pt], 1.0)
        opt.step()
        sch.step()
        g.copy_(grad)
        ops.sqnorm(g, sq, 1.0, lazy=(lo, hi))
        ops.adamw_step(p, g, m, v, pb, sq, step, hyper, 1.0, lazy=(lo, hi), lazy_decay=lazy_decay)
        ops.advance_counters(step, rng(), sq)
        assert torch.equal(p[lo:hi], p0[lo:hi]) and torch.all(m[lo:hi] == 0) and torch.all(v[lo:hi] == 0)
    p[lo:hi] *= lazy_decay
    torch.testing.assert_close(p, pt.detach(), rtol=1e-5, atol=1e-6)
    assert torch.equal(pb[:lo], p[:lo].bfloat16()) and torch.equal(pb[hi:], p[hi:].bfloat16())


# ------------------------------------------------------------------ diffusion / data
def test_ddim_step():
    x = torch.randn(64, 3, 64, 64, device=DEV)
    x0 = torch.randn_like(x) * 2
    c = ref.ddim_coeffs(2000, 1999, 20)
    coef = torch.tensor(c, device=DEV)
    xn, x0c = ops.ddim_step(x, x0, coef)
    xr, x0r = ref.ddim_step(x, x0, c)
    close(xn, xr, 1e-4, 1e-5, "x_next")
    close(x0c, x0r, 0, 0, "x0")


def test_randn_stats():
    out = torch.empty(1_000_001, device=DEV)
    ops.randn_(out, rng(), 3)
    assert abs(out.mean().item()) < 5e-3
    assert abs(out.std().item() - 1) < 5e-3
    out2 = torch.empty(1001, device=DEV)
    ops.randn_(out2, rng(), 3)
    cpu = torch.empty(1001)
    ops.randn_(cpu, rng().cpu(), 3)
    close(out2.cpu(), cpu, 1e-4, 1e-4, "randn hip vs cpu")


@pytest.mark.parametrize("H", [64, 200, 32])
def test_pixelate_pair(H):
    B = 6
    img = torch.randn(B, 3, H, H, device=DEV)
    t = torch.tensor([1, 2, 3, 4, 5, 6 if H >= 64 else 5], device=DEV)
    xt, xtm1 = ops.pixelate_pair(img, None, t, B)
    for i in range(B):
        close(xt[i:i + 1], ref.pixelate(img[i:i + 1], 2 ** int(t[i])), 0, 0, "x_t")
        close(xtm1[i:i + 1], ref.pixelate(img[i:i + 1], 2 ** (int(t[i]) - 1)), 0, 0, "x_t-1")


def test_cold_batch_and_q_sample():
    pool = torch.randn(50, 3, 64, 64, device=DEV)
    B = 32
    xt, xtm1 = torch.empty(B, 3, 64, 64, device=DEV), torch.empty(B, 3, 64, 64, device=DEV)
    t, idx = torch.empty(B, dtype=torch.int64, device=DEV), torch.empty(B, dtype=torch.int64, device=DEV)
    ops.cold_batch(pool, rng(), 2, xt, xtm1, t, idx, 6)
    assert t.min().item() >= 1 and t.max().item() <= 6
    a, b = ops.pixelate_pair(pool, idx, t, B)
    close(xt, a, 0, 0, "cold x_t")
    close(xtm1, b, 0, 0, "cold x_t-1")
    x0 = torch.randn(B, 3, 8, 8, device=DEV)
    eps = torch.randn_like(x0)
    tt = torch.randint(0, 2000, (B,), device=DEV)
    close(ops.q_sample(x0, tt, eps, 2000), ref.q_sample(x0, tt, eps, 2000), 1e-5, 1e-5, "q_sample")
