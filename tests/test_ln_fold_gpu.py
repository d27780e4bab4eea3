"""LayerNorm fold kernels (csrc/gemm.hip fold epilogues, ln_fold_kernel, the
patch-embed / residual producers and the LayerNorm backward's output re-emission)
vs the plain-PyTorch fp32 reference (ddim_cold_amd/ops/reference.py)."""
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
    bad = (~(err <= atol + rtol * b.abs())).sum().item()  # NaN counts as a mismatch
    assert bad == 0, f"{name}: {bad} mismatches, max err {err.max().item():.3e}"


def folded(Nout, K, M, shift=0.5, scale=2.0):
    """Raw rows x (fp32 + bf16 copy + stats) and LayerNorm-folded weights."""
    x = torch.randn(M, K, device=DEV) * scale + shift
    st = ref.row_stats(x)
    w = torch.randn(Nout, K, device=DEV) * 0.05
    g, be = torch.randn(K, device=DEV), torch.randn(K, device=DEV)
    b = torch.randn(Nout, device=DEV)
    wf = torch.empty(Nout, K, dtype=torch.bfloat16, device=DEV)
    c, bf = torch.empty(Nout, device=DEV), torch.empty(Nout, device=DEV)
    ops.ln_fold_([w], [g], [be], [b], [wf], [c], [bf])
    return x, x.to(torch.bfloat16), st, w, g, be, b, wf, c, bf


@pytest.mark.parametrize("rows,K", [(1152, 384), (384, 384), (192, 384), (768, 256), (20, 64)])
def test_ln_fold_kernel(rows, K):
    w = torch.randn(rows, K, device=DEV)
    g, be, b = torch.randn(K, device=DEV), torch.randn(K, device=DEV), torch.randn(rows, device=DEV)
    outs = [torch.empty(rows, K, dtype=torch.bfloat16, device=DEV), torch.empty(rows, device=DEV),
            torch.empty(rows, device=DEV)]
    ops.ln_fold_([w], [g], [be], [b], *[[o] for o in outs])
    exp = [torch.empty_like(o) for o in outs]
    ref.ln_fold(w, g, be, b, *exp)
    close(outs[0], exp[0], 0, 0, "wf")
    close(outs[1], exp[1], 1e-3, 1e-5, "c")
    close(outs[2], exp[2], 1e-3, 1e-5, "bf")


@pytest.mark.parametrize("n", [16, 25])
def test_ln_fold_kernel_many(n):
    """n GEMMs of different row counts in one launch (the model's table: 15 for ViT-tiny,
    25 for vit_small_200)."""
    K = 128
    jobs = [(torch.randn(r, K, device=DEV), torch.randn(K, device=DEV), torch.randn(K, device=DEV),
             torch.randn(r, device=DEV) if i % 3 else None) for i, r in enumerate(([384, 128, 40, 8] * 7)[:n])]
    outs = [(torch.empty(w.shape[0], K, dtype=torch.bfloat16, device=DEV), torch.empty(w.shape[0], device=DEV),
             torch.empty(w.shape[0], device=DEV)) for w, _, _, _ in jobs]
    ops.ln_fold_(*[list(z) for z in zip(*jobs)], *[list(z) for z in zip(*outs)])
    for (w, g, be, b), (wf, c, bf) in zip(jobs, outs):
        e = [torch.empty_like(wf), torch.empty_like(c), torch.empty_like(bf)]
        ref.ln_fold(w, g, be, b, *e)
        close(wf, e[0], 0, 0, "wf")
        close(bf, e[2], 1e-3, 1e-5, "bf")


@pytest.mark.parametrize("B,N,H,D", [(32, 65, 12, 384), (4, 257, 4, 256), (3, 17, 2, 128)])
def test_qkv_fold(B, N, H, D):
    M = B * N
    x, xb, st, w, g, be, b, wf, c, bf = folded(3 * D, D, M)
    mean, rstd = torch.empty(M, device=DEV), torch.empty(M, device=DEV)
    out = ops.qkv_fwd(xb, wf, bf, B, N, H, fold=(st, c, 1e-5, mean, rstd))
    outr = ref.qkv_fwd(xb, wf, bf, B, N, H, st, c, 1e-5)
    close(out, outr, 2e-2, 1e-2, "qkv fold")
    close(mean, x.mean(-1), 1e-4, 1e-4, "mean")
    close(rstd, torch.rsqrt(x.var(-1, unbiased=False) + 1e-5), 1e-4, 1e-3, "rstd")
    # against the unfolded math: LayerNorm -> bf16 -> GEMM (bf16 operands of different rounding)
    ln = torch.nn.functional.layer_norm(x, (D,), g, be, 1e-5)
    yr = (ln @ w.t() + b).view(B, N, 3, H, D // H).permute(2, 0, 3, 1, 4)
    close(out, yr, 6e-2, 3e-2, "qkv vs LayerNorm+GEMM")


def test_gelu_and_linear_fold():
    M, K, Hm = 2080, 384, 384
    x, xb, st, w, g, be, b, wf, c, bf = folded(Hm, K, M)
    r = rng()
    mean, rstd = torch.empty(M, device=DEV), torch.empty(M, device=DEV)
    u, h = ops.linear_gelu_fwd(xb, wf, bf, r, 9, 0.1, fold=(st, c, 1e-5, mean, rstd))
    ur, hr = ref.linear_gelu_fwd(xb, wf, bf, r, 9, 0.1, st, c, 1e-5)
    close(u, ur, 2e-2, 1e-2, "u")
    close(h, hr, 2e-2, 1e-2, "h")
    close(mean, x.mean(-1), 1e-4, 1e-4, "mean")
    for f32 in (True, False):
        y = ops.linear_fwd(xb, wf, bf, f32, fold=(st, c, 1e-5))
        yr = ref.linear_fwd(xb, wf, bf, f32, st, c, 1e-5)
        close(y, yr, 2e-2 if not f32 else 2e-3, 1e-2 if not f32 else 1e-3, f"linear fold f32={f32}")


@pytest.mark.parametrize("B,C,H,W,p,D", [(4, 3, 64, 64, 8, 384), (2, 3, 64, 64, 4, 256)])
def test_head_fold(B, C, H, W, p, D):
    N = (H // p) * (W // p) + 1
    M = B * N
    x, xb, st, w, g, be, b, wf, c, bf = folded(C * p * p, D, M)
    mean, rstd = torch.full((M,), float("nan"), device=DEV), torch.full((M,), float("nan"), device=DEV)
    img = ops.head_fwd(xb, wf, bf, B, C, H, W, p, fold=(st, c, 1e-5, mean, rstd))
    imgr = ref.head_fwd(xb, wf, bf, B, C, H, W, p, st, c, 1e-5)
    close(img, imgr, 2e-3, 1e-3, "head fold")
    # every row's statistics are written, cls rows (skipped by the head epilogue) included
    assert torch.isfinite(mean).all() and torch.isfinite(rstd).all()
    close(mean, x.mean(-1), 1e-4, 1e-4, "mean")
    xk = torch.randn(B, C, H, W, device=DEV)
    ops.head_step_(xb, wf, bf, xk, None, None, p, 2, fold=(st, c, 1e-5))
    close(xk, imgr.clamp(-1, 1), 2e-3, 1e-3, "head_step fold")


@pytest.mark.parametrize("M,K,Nout,pd,pdp", [(2080, 384, 384, 0.1, 0.1), (100, 64, 64, 0.0, 0.3),
                                              (4160, 384, 384, 0.0, 0.0), (8224, 256, 256, 0.1, 0.0)])
def test_residual_producer_stats(M, K, Nout, pd, pdp):
    N = 65 if M % 65 == 0 else (257 if M % 257 == 0 else 25)
    a = (torch.randn(M, K, device=DEV)).to(torch.bfloat16)
    w = (torch.randn(Nout, K, device=DEV) * 0.05).to(torch.bfloat16)
    b = torch.randn(Nout, device=DEV)
    x = torch.randn(M, Nout, device=DEV)
    r = rng()
    st = torch.full((M, Nout // 32, 2), float("nan"), device=DEV)  # every slot must be written
    xb = torch.empty(M, Nout, dtype=torch.bfloat16, device=DEV)
    y = ops.linear_residual_fwd(a, w, b, x, N, r, 3, pd, 4, pdp, st_out=st, xb_out=xb)
    yr = ref.linear_residual_fwd(a, w, b, x, N, r, 3, pd, 4, pdp)
    close(y, yr, 1e-3, 1e-4, "resid")
    close(xb, y.to(torch.bfloat16), 0, 0, "bf16 copy")
    close(st, ref.row_stats(y), 1e-3, 1e-4, "row statistics slots")
    # deterministic: a second run writes bit-identical statistics
    st2 = torch.empty_like(st)
    ops.linear_residual_fwd(a, w, b, x, N, r, 3, pd, 4, pdp, st_out=st2, xb_out=xb)
    assert torch.equal(st, st2)


@pytest.mark.parametrize("B,C,H,W,p,D,pd", [(4, 3, 64, 64, 8, 384, 0.1), (2, 3, 64, 64, 4, 256, 0.0)])
def test_patch_embed_producer_stats(B, C, H, W, p, D, pd):
    N = (H // p) * (W // p) + 1
    M = B * N
    img = torch.randn(B, C, H, W, device=DEV)
    t = torch.randint(0, 2000, (B,), device=DEV)
    w = (torch.randn(D, C * p * p, device=DEV) * 0.05).to(torch.bfloat16)
    b, cls, pos = torch.randn(D, device=DEV), torch.randn(D, device=DEV), torch.randn(N, D, device=DEV)
    temb = torch.randn(2000, D, device=DEV)
    r = rng()
    st = torch.full((M, D // 32, 2), float("nan"), device=DEV)  # every slot must be written
    xb = torch.empty(M, D, dtype=torch.bfloat16, device=DEV)
    x, _ = ops.patch_embed_fwd(img, t, w, b, cls, pos, temb, r, 1, pd, p, ln_st=st, xb_out=xb)
    xr, _ = ref.patch_embed_fwd(img, t, w, b, cls, pos, temb, r, 1, pd, p)
    x2 = x.view(M, D)
    close(x, xr, 1e-3, 1e-3, "tokens")
    close(xb, x2.to(torch.bfloat16), 0, 0, "bf16 copy")
    # patch rows: per-slot sums; cls rows: the whole row in slot 0
    stn = st.view(B, N, D // 32, 2)
    exp = ref.row_stats(x2).view(B, N, D // 32, 2)
    close(stn[:, 1:], exp[:, 1:], 1e-3, 1e-4, "patch-row slots")
    close(stn[:, 0].sum(1), exp[:, 0].sum(1), 1e-3, 1e-4, "cls-row totals")


def test_layernorm_bwd_emits_output():
    M, D, N = 2080, 384, 65
    x = torch.randn(M, D, device=DEV) * 2 + 0.3
    g, be = torch.randn(D, device=DEV), torch.randn(D, device=DEV)
    yr, mu, rs = ref.layernorm_fwd(x, g, be)
    dy = torch.randn(M, D, device=DEV)
    dg, db = torch.zeros(D, device=DEV), torch.zeros(D, device=DEV)
    y = torch.empty(M, D, dtype=torch.bfloat16, device=DEV)
    go, _ = ops.layernorm_bwd(dy, x, mu, rs, g, None, dg, db, N, rng(), 0, 0.0, 0, 0.0, False, beta=be, y_out=y)
    gor, _ = ref.layernorm_bwd(dy, x, mu, rs, g, None, torch.zeros(D, device=DEV), torch.zeros(D, device=DEV),
                               N, rng(), 0, 0.0, 0, 0.0, False)
    close(go, gor, 1e-4, 1e-4, "g_out")
    close(y, yr, 2e-2, 1e-2, "LayerNorm output")


def test_folded_program_matches_unfolded():
    """Whole ViT-tiny forward (train mode, dropout on) with and without the fold."""
    from ddim_cold_amd.models import build_model
    from ddim_cold_amd.models import program as pr
    m = build_model("vit_tiny").to(DEV).train()
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "norm" in n:
                p.add_(0.2 * torch.randn_like(p))
    prog = m.program()
    img = torch.randn(8, 3, 64, 64, device=DEV)
    t = torch.randint(0, 2000, (8,), device=DEV)
    r = rng()
    P = pr.model_tensors(m)
    assert P.folded
    a, _ = prog.forward(P, img, t, r, True)
    Pu = pr.collect({n: (pr._bf16_cached(m, n, p) if pr.is_matrix_param(n) else p.detach())
                     for n, p in m.named_parameters()}, prog.cfg.depth, prog.cfg.dim)
    b, _ = prog.forward(Pu, img, t, r, True)
    rel = (a - b).abs().max().item() / b.abs().max().item()
    assert rel < 3e-2, rel


@pytest.mark.parametrize("splits", [1, 2, 3])
def test_bf16_dgrad_into_layernorm_bwd(splits):
    """bf16 input-gradient GEMM (optionally K-split into bf16 partials) feeding the
    LayerNorm backward, which sums the partials in fp32."""
    M, Nout, K, N = 2080, 1152, 384, 65
    dy = (torch.randn(M, Nout, device=DEV)).to(torch.bfloat16)
    w = (torch.randn(Nout, K, device=DEV) * 0.05).to(torch.bfloat16)
    parts = ops.linear_dgrad(dy, w, False, splits)
    pr = ref.linear_dgrad(dy, w, False, splits)
    assert parts.dtype == torch.bfloat16 and parts.shape == pr.shape
    close(parts, pr, 2e-2, 1e-2, "bf16 dgrad partials")
    x = torch.randn(M, K, device=DEV) * 2 + 0.3
    g, be = torch.randn(K, device=DEV), torch.randn(K, device=DEV)
    _, mu, rs = ref.layernorm_fwd(x, g, be)
    dg1, db1, dg2, db2 = (torch.zeros(K, device=DEV) for _ in range(4))
    go, gy = ops.layernorm_bwd(parts, x, mu, rs, g, None, dg1, db1, N, rng(), 7, 0.1, 8, 0.1, True)
    gor, gyr = ref.layernorm_bwd(parts, x, mu, rs, g, None, dg2, db2, N, rng(), 7, 0.1, 8, 0.1, True)
    close(go, gor, 1e-4, 1e-4, "g_out")
    close(dg1, dg2, 1e-2, 1e-4, "dgamma")
    close(db1, db2, 1e-2, 1e-4, "dbeta")
    close(gy, gyr, 1e-2, 1e-2, "gy")


@pytest.mark.parametrize("B,C,H,W,p,D,fold", [(32, 3, 64, 64, 8, 384, True), (4, 3, 64, 64, 4, 256, False),
                                              (3, 3, 32, 32, 8, 128, True)])
def test_head_loss_fused(B, C, H, W, p, D, fold):
    """Head GEMM with the smooth-L1 loss + token-layout gradient in its epilogue ==
    head_fwd + smooth_l1_fwd_bwd."""
    N = (H // p) * (W // p) + 1
    M = B * N
    F = C * p * p
    if fold:
        x, a, st, w, g, be, b, wf, c, bf = folded(F, D, M)
        fk = (st, c, 1e-5)
    else:
        a = torch.randn(M, D, device=DEV).to(torch.bfloat16)
        wf = (torch.randn(F, D, device=DEV) * 0.05).to(torch.bfloat16)
        bf = torch.randn(F, device=DEV) * 0.1
        fk = None
    target = torch.randn(B, C, H, W, device=DEV).clamp(-1, 1)
    parts, dtok = ops.head_loss(a, wf, bf, target, p, 1.0, fold=fk)
    img = ops.head_fwd(a, wf, bf, B, C, H, W, p, fold=fk)
    loss_r, dtok_r = ops.smooth_l1_fwd_bwd(img, target, N, p, 1.0)
    torch.testing.assert_close(parts.sum(), loss_r.reshape(()), rtol=1e-4, atol=1e-6)
    close(dtok, dtok_r, 1e-6, 1e-2, "token-layout gradient")
    assert torch.count_nonzero(dtok.view(B, N, F)[:, 0]) == 0


def test_ln_fold_kernel_bf16_weights():
    """Fold from the optimizer's bf16 weight shadow (what the train engine does)."""
    rows, K = 1152, 384
    w = (torch.randn(rows, K, device=DEV)).to(torch.bfloat16)
    g, be, b = torch.randn(K, device=DEV), torch.randn(K, device=DEV), torch.randn(rows, device=DEV)
    outs = [torch.empty(rows, K, dtype=torch.bfloat16, device=DEV), torch.empty(rows, device=DEV),
            torch.empty(rows, device=DEV)]
    ops.ln_fold_([w], [g], [be], [b], *[[o] for o in outs])
    exp = [torch.empty_like(o) for o in outs]
    ref.ln_fold(w.float(), g, be, b, *exp)
    close(outs[0], exp[0], 0, 0, "wf")
    close(outs[1], exp[1], 1e-3, 1e-5, "c")
    close(outs[2], exp[2], 1e-3, 1e-5, "bf")
