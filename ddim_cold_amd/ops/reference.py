"""Pure-PyTorch reference implementations of every fused op.

Each function here has exactly the signature and numerics contract of the
HIP op of the same name in ``csrc/`` (registered as ``torch.ops.ddim_cold.*``):
same output dtypes (bf16 activations, fp32 residual stream / statistics /
gradients), same rounding points, and the same counter-based dropout masks
(``keep_mask`` below is bit-identical to ``dropout_keep`` in
``csrc/common.h``).  They serve three purposes:

1. oracle for the kernel numerics tests (``tests/test_kernels_gpu.py``),
2. the CPU backend of the fused program (so the program logic — the
   hand-written backward, masks, gradient layout — is unit-tested on CPU
   against autograd of :meth:`DiffusionVisionTransformer.forward_reference`),
3. documentation of the op contracts.

Tensor conventions: ``M = B*N`` token rows (N = P+1 tokens incl. cls),
``D`` embed dim, ``F = C*p*p`` pixels per patch, weights in nn.Linear
layout ``[out, in]`` and their transposes ``[in, out]`` for dgrad.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn.functional as F

MASK32 = 0xFFFFFFFF
GOLDEN = 0x9E3779B1
SALT_C1 = 0x9E3779B9
SALT_C2 = 0x85EBCA6B


# ----------------------------------------------------------------------------- RNG
def _mul32(x, c: int):
    """(x * c) mod 2^32 for int64 tensors / python ints holding uint32 values."""
    if isinstance(x, int):
        return (x * c) & MASK32
    lo = x * (c & 0xFFFF)
    hi = (x * (c >> 16)) & 0xFFFF
    return (lo + (hi << 16)) & MASK32


def mix32(x):
    """lowbias32 integer hash (bijective on uint32)."""
    x = x ^ (x >> 16)
    x = _mul32(x, 0x7FEB352D)
    x = x ^ (x >> 15)
    x = _mul32(x, 0x846CA68B)
    x = x ^ (x >> 16)
    return x


def site_salt(rng: torch.Tensor, site: int) -> int:
    """Per-(step, dropout-site) salt from the device RNG state ``rng = [seed, step]``."""
    seed, step = (int(v) for v in rng.detach().cpu().tolist())
    s_lo, s_hi = seed & MASK32, (seed >> 32) & MASK32
    a = mix32((_mul32(step & MASK32, SALT_C1) + s_hi) & MASK32)
    b = mix32(s_lo ^ a)
    return mix32((b + _mul32(site & MASK32, SALT_C2)) & MASK32)


DROP_MUL1 = 0xED5AD5
DROP_MUL2 = 0x2C1B3D


def drop_mix(x):
    """Dropout pair hash (csrc/common.h ``drop_mix``): xorshift-multiply rounds with
    24-bit multipliers (full-rate ``v_mul_u32_u24`` on gfx950)."""
    x = x ^ (x >> 16)
    x = ((x & 0xFFFFFF) * DROP_MUL1) & MASK32
    x = x ^ (x >> 16)
    x = ((x & 0xFFFFFF) * DROP_MUL2) & MASK32
    x = x ^ (x >> 16)
    return x


def drop_threshold(p: float) -> int:
    """Drop iff the element's 16-bit hash half < threshold; threshold = 2 round(p * 2^15)
    (even: the attention forward compares the halves shifted right by one)."""
    v = p * 32768.0 + 0.5
    return 65536 if v >= 32768.0 else 2 * max(int(v), 0)


def keep_mask(numel: int, rng: torch.Tensor, site: int, p: float, device=None, start: int = 0) -> torch.Tensor:
    """Boolean keep-mask over a flat index space [start, start + numel) (bit-exact with
    ``dropout_keep`` in csrc/common.h): element i uses the 16-bit half (i & 1) of the
    hash of pair i >> 1 (indices are 32-bit counters)."""
    salt = site_salt(rng, site)
    idx = torch.arange(start, start + numel, dtype=torch.int64, device=device) & MASK32
    h = drop_mix((_mul32(idx >> 1, GOLDEN) + salt) & MASK32)
    half = torch.where((idx & 1) == 1, h >> 16, h & 0xFFFF)
    return half >= drop_threshold(p)


def attn_mask_ld(N: int) -> int:
    """Row stride of the attention-probability mask index (csrc/common.h attn_mask_ld)."""
    return (N + 3) // 4 * 4


def attn_keep_mask(B: int, H: int, N: int, rng, site: int, p: float, device=None, bh0: int = 0) -> torch.Tensor:
    """[B, H, N, N] keep-mask of the attention probabilities; element (b, h, q, key) has
    flat index ((bh0 + b*H + h)*N + q) * attn_mask_ld(N) + key (``bh0``: the first
    head's position in a larger batch, for checking a slice of one)."""
    ld = attn_mask_ld(N)
    return keep_mask(B * H * N * ld, rng, site, p, device, start=bh0 * N * ld).view(B, H, N, ld)[..., :N]


def _dropout(x: torch.Tensor, rng, site, p) -> torch.Tensor:
    if p <= 0.0:
        return x
    m = keep_mask(x.numel(), rng, site, p, x.device).view(x.shape)
    return torch.where(m, x / (1.0 - p), torch.zeros((), dtype=x.dtype, device=x.device))


def _sample_scale(B: int, rng, site, p, device) -> torch.Tensor:
    """DropPath per-sample scale (0 or 1/(1-p)); shape [B]."""
    if p <= 0.0:
        return torch.ones(B, device=device)
    m = keep_mask(B, rng, site, p, device)
    return m.float() / (1.0 - p)


def bf16(x: torch.Tensor) -> torch.Tensor:
    return x.to(torch.bfloat16)


def _mm(a: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """fp32-accumulated ``a @ w.T`` on bf16 inputs."""
    return a.float() @ w.float().t()


def gelu(x):
    return 0.5 * x * (1.0 + torch.erf(x * 0.7071067811865476))


def gelu_grad(x):
    cdf = 0.5 * (1.0 + torch.erf(x * 0.7071067811865476))
    pdf = torch.exp(-0.5 * x * x) * 0.3989422804014327
    return cdf + x * pdf


# ----------------------------------------------------------------------------- forward ops
def patchify_bf16(img: torch.Tensor, patch: int) -> torch.Tensor:
    """[B,C,H,W] fp32 -> conv-im2col rows [B*P, C*p*p] bf16 (k = c*p*p + i*p + j)."""
    B, C, H, W = img.shape
    Hp, Wp = H // patch, W // patch
    t = img.reshape(B, C, Hp, patch, Wp, patch).permute(0, 2, 4, 1, 3, 5)
    return bf16(t.reshape(B * Hp * Wp, C * patch * patch))


LN_SLOT = 32  # csrc/gemm.hip: row statistics per 32-column slot


def row_stats(x: torch.Tensor) -> torch.Tensor:
    """LayerNorm-fold row statistics [M, D/32, 2]: {sum, sum^2} of each row's 32-column slots."""
    D = x.shape[-1]
    xf = x.reshape(-1, D // LN_SLOT, LN_SLOT).float()
    return torch.stack((xf.sum(-1), (xf * xf).sum(-1)), dim=-1)


def _row_stats_add_(st: torch.Tensor, x: torch.Tensor):
    """Write the LayerNorm-fold producer statistics of ``x`` into ``st`` ([M, D/32, 2])."""
    st.copy_(row_stats(x).view(st.shape))


def patch_embed_fwd(img, t, w_pe, b_pe, cls, pos, temb, rng, site: int, p: float, patch: int, ln_st=None,
                    xb_out=None):
    """tokens x[B,N,D] fp32 = pos_drop(cat(cls, conv(img)) + pos + temb[t]); also the bf16 patches.
    LayerNorm fold: ``ln_st`` [B*N, D/32, 2] = the tokens' row statistics
    (:func:`row_stats`); ``xb_out`` = the tokens in bf16."""
    B = img.shape[0]
    D = w_pe.shape[0]
    patches = patchify_bf16(img, patch)
    proj = _mm(patches, w_pe.reshape(D, -1)) + b_pe.float()
    proj = proj.view(B, -1, D)
    tok = torch.cat((cls.float().reshape(1, 1, D).expand(B, 1, D), proj), dim=1)
    tok = tok + pos.float().reshape(1, -1, D) + temb.float()[t].unsqueeze(1)
    tok = _dropout(tok, rng, site, p).contiguous()
    if ln_st is not None:
        _row_stats_add_(ln_st, tok)
        xb_out.copy_(bf16(tok).view(xb_out.shape))
    return tok, patches


def layernorm_fwd(x, gamma, beta, eps: float = 1e-5):
    xf = x.float()
    mean = xf.mean(-1)
    var = ((xf - mean.unsqueeze(-1)) ** 2).mean(-1)
    rstd = torch.rsqrt(var + eps)
    y = (xf - mean.unsqueeze(-1)) * rstd.unsqueeze(-1) * gamma.float() + beta.float()
    return bf16(y), mean, rstd


def ln_row_stats(st: torch.Tensor, K: int, eps: float):
    """(mean, rstd) of rows from their per-slot {sum, sum^2} ([M, K/32, 2]; LayerNorm fold)."""
    tot = st.reshape(st.shape[0], -1, 2).sum(1)
    mu = tot[:, 0] / K
    var = torch.clamp(tot[:, 1] / K - mu * mu, min=0.0)
    return mu, torch.rsqrt(var + eps)


def _lin(a, w, b, st=None, c=None, eps: float = 1e-5, mean_out=None, rstd_out=None):
    """fp32 ``a @ w.T + b``; with the LayerNorm fold (``st`` = row {sum, sum^2} of the
    raw rows ``a``, ``w``/``b``/``c`` from :func:`ln_fold`):
    ``rstd * (a @ w.T - mean * c) + b`` = LayerNorm(a) @ W.T + bias."""
    a2 = a.reshape(-1, a.shape[-1])
    y = _mm(a2, w)
    if st is not None:
        mu, rs = ln_row_stats(st.reshape(a2.shape[0], -1, 2), a2.shape[1], eps)
        y = (y - mu.unsqueeze(1) * c.float().unsqueeze(0)) * rs.unsqueeze(1)
        if mean_out is not None:
            mean_out.copy_(mu.view(mean_out.shape))
            rstd_out.copy_(rs.view(rstd_out.shape))
    if b is not None:
        y = y + b.float()
    return y


def linear_fwd(a, w, b, out_fp32: bool, st=None, c=None, eps: float = 1e-5):
    y = _lin(a, w, b, st, c, eps)
    return y if out_fp32 else bf16(y)


def qkv_fwd(a, w, b, B: int, N: int, H: int, st=None, c=None, eps: float = 1e-5, mean_out=None, rstd_out=None):
    """QKV projection written head-major: [3, B, H, N, hd] bf16."""
    D3 = w.shape[0]
    D = D3 // 3
    y = bf16(_lin(a, w, b, st, c, eps, mean_out, rstd_out))
    return y.view(B, N, 3, H, D // H).permute(2, 0, 3, 1, 4).contiguous()


def attn_fwd(qkv, scale: float, rng, site: int, p: float, bh0: int = 0):
    """softmax(QK^T*scale) (dropout) V -> o [B,N,D] bf16 token-major, lse [B,H,N] fp32."""
    _, B, H, N, hd = qkv.shape
    q, k, v = qkv[0].float(), qkv[1].float(), qkv[2].float()
    s = (q @ k.transpose(-1, -2)) * scale
    lse = torch.logsumexp(s, dim=-1)
    pr = torch.exp(s - lse.unsqueeze(-1))
    if p > 0.0:
        pr = torch.where(attn_keep_mask(B, H, N, rng, site, p, pr.device, bh0), pr / (1.0 - p),
                         torch.zeros((), dtype=pr.dtype, device=pr.device))
    # P is rounded to bf16 before the PV product (as the MFMA kernel does)
    o = bf16(pr).float() @ v
    return bf16(o.transpose(1, 2).reshape(B, N, H * hd)), lse


def linear_residual_fwd(a, w, b, x, N: int, rng, site_drop: int, p_drop: float,
                        site_dp: int, p_dp: float, st_out=None, xb_out=None):
    """x_new = x + DropPath(Dropout(a @ w.T + b)) (fp32 residual stream); LayerNorm-fold
    producer: st_out = row statistics of x_new (:func:`row_stats`), xb_out = bf16(x_new)."""
    M, Dout = x.shape[0] * (x.shape[1] if x.dim() == 3 else 1), w.shape[0]
    y = _mm(a.reshape(-1, a.shape[-1]), w) + b.float()
    y = _dropout(y, rng, site_drop, p_drop)
    B = M // N
    sc = _sample_scale(B, rng, site_dp, p_dp, x.device).repeat_interleave(N)
    out = (x.reshape(M, Dout).float() + y * sc.unsqueeze(1)).view(x.shape)
    if st_out is not None:
        _row_stats_add_(st_out, out)
        xb_out.copy_(bf16(out).view(xb_out.shape))
    return out


def linear_gelu_fwd(a, w, b, rng, site: int, p: float, st=None, c=None, eps: float = 1e-5, mean_out=None,
                    rstd_out=None):
    """u = a @ w.T + b (bf16, saved); h = Dropout(GELU(u)) (bf16)."""
    u = _lin(a, w, b, st, c, eps, mean_out, rstd_out)
    u16 = bf16(u)
    h = _dropout(gelu(u), rng, site, p)
    return u16, bf16(h)


def head_fwd(a, w, b, B: int, C: int, H: int, W: int, patch: int, st=None, c=None, eps: float = 1e-5,
             mean_out=None, rstd_out=None):
    """Head linear on patch tokens, unpatchified straight to [B,C,H,W] fp32."""
    N = a.shape[0] // B
    y = _lin(a, w, b, st, c, eps, mean_out, rstd_out).view(B, N, -1)[:, 1:, :]
    Hp, Wp = H // patch, W // patch
    img = y.reshape(B, Hp, Wp, patch, patch, C).permute(0, 5, 1, 3, 2, 4)
    return img.reshape(B, C, H, W).contiguous()


def img_to_tokgrad(dimg, N: int, patch: int):
    """[B,C,H,W] grad -> token-layout [B*N, C*p*p] bf16 (cls rows zero)."""
    B, C, H, W = dimg.shape
    Hp, Wp = H // patch, W // patch
    t = dimg.float().reshape(B, C, Hp, patch, Wp, patch).permute(0, 2, 4, 3, 5, 1)
    t = t.reshape(B, Hp * Wp, patch * patch * C)
    out = torch.zeros(B, N, patch * patch * C, device=dimg.device)
    out[:, 1:, :] = t
    return bf16(out.reshape(B * N, -1))


def smooth_l1_fwd_bwd(pred, target, N: int, patch: int, beta: float = 1.0):
    """mean smooth-L1 loss and its grad in token layout (bf16, cls rows zero)."""
    d = pred.float() - target.float()
    ad = d.abs()
    loss = torch.where(ad < beta, 0.5 * d * d / beta, ad - 0.5 * beta).mean()
    g = torch.clamp(d / beta, -1.0, 1.0) / d.numel()
    return loss.reshape(1), img_to_tokgrad(g, N, patch)


# ----------------------------------------------------------------------------- backward ops
def linear_dgrad(dy, w, out_fp32: bool, splits: int = 1):
    """dx = dy @ W  (W in nn.Linear layout [N_out, K]).  ``splits`` > 1: the
    [splits, M, K] partial products over 64-aligned slices of N_out, as the
    K-split kernel writes them (their sum is dx; fp32 or bf16 each)."""
    if splits > 1:
        kt = (dy.shape[1] + 63) // 64
        step = (kt + splits - 1) // splits * 64
        parts = torch.stack([dy[:, z * step:(z + 1) * step].float() @ w[z * step:(z + 1) * step].float()
                             for z in range(splits)])
        return parts if out_fp32 else bf16(parts)
    dx = dy.float() @ w.float()
    return dx if out_fp32 else bf16(dx)


def linear_dgrad_gelu(dy, w, u, rng, site: int, p: float):
    """du = Dropout(dy @ W) * GELU'(u)  (mask of the post-GELU dropout)."""
    dh = dy.float() @ w.float()
    dh = _dropout(dh, rng, site, p)
    return bf16(dh * gelu_grad(u.float()))


def linear_wgrad(dy, x, dw, db: Optional[torch.Tensor]):
    """dw += dy^T @ x ; db += colsum(dy)  (fp32 accumulate, in place)."""
    dw.add_((dy.float().t() @ x.float()).view_as(dw))
    if db is not None:
        db.add_(dy.float().sum(0))


def layernorm_out_(x, mean, rstd, gamma, beta, y_out):
    """y_out = bf16((x - mean) * rstd * gamma + beta) (LayerNorm output from saved statistics)."""
    D = x.shape[-1]
    xf = x.reshape(-1, D).float()
    y = (xf - mean.reshape(-1, 1)) * rstd.reshape(-1, 1) * gamma.float() + beta.float()
    y_out.copy_(bf16(y).view(y_out.shape))


def ln_fold(w, gamma, beta, bias, wf, c, bf):
    """LayerNorm fold weights: wf = bf16(gamma o W); c = rowsum(wf) (of the bf16
    values); bf = bias + W beta.  ``w`` fp32, or its bf16 copy (then used as is)."""
    wq = bf16(w.float() * gamma.float().unsqueeze(0))
    wf.copy_(wq.view(wf.shape))
    c.copy_(wq.float().sum(1).view(c.shape))
    bb = w.float() @ beta.float()
    if bias is not None:
        bb = bb + bias.float()
    bf.copy_(bb.view(bf.shape))


def layernorm_bwd(dy, x, mean, rstd, gamma, g_res, dgamma, dbeta, N: int, rng,
                  site_drop: int, p_drop: float, site_dp: int, p_dp: float, emit_gy: bool):
    """g_out = g_res + LN^T(dy);  dgamma/dbeta += ...;  gy = bf16(g_out * branch masks)."""
    M, D = x.shape[0] * (x.shape[1] if x.dim() == 3 else 1), x.shape[-1]
    xf = x.reshape(M, D).float()
    dyf = dy.reshape(-1, M, D).float().sum(0)  # K-split dgrad partials summed
    xhat = (xf - mean.reshape(M, 1)) * rstd.reshape(M, 1)
    dgamma.add_((dyf * xhat).sum(0))
    dbeta.add_(dyf.sum(0))
    dxh = dyf * gamma.float()
    dx = (dxh - dxh.mean(-1, keepdim=True) - xhat * (dxh * xhat).mean(-1, keepdim=True)) * rstd.reshape(M, 1)
    g_out = dx if g_res is None else g_res.reshape(M, D).float() + dx
    gy = None
    if emit_gy:
        z = _dropout(g_out, rng, site_drop, p_drop)
        B = M // N
        sc = _sample_scale(B, rng, site_dp, p_dp, x.device).repeat_interleave(N)
        gy = bf16(z * sc.unsqueeze(1))
    return g_out.view(x.shape), gy


def attn_bwd(do, qkv, o, lse, scale: float, rng, site: int, p: float, bh0: int = 0):
    """Flash-style attention backward -> dqkv [B*N, 3D] bf16 token-major."""
    _, B, H, N, hd = qkv.shape
    q, k, v = qkv[0].float(), qkv[1].float(), qkv[2].float()
    dof = do.float().view(B, N, H, hd).transpose(1, 2)  # [B,H,N,hd]
    of = o.float().view(B, N, H, hd).transpose(1, 2)
    s = (q @ k.transpose(-1, -2)) * scale
    pr = torch.exp(s - lse.unsqueeze(-1))
    if p > 0:
        m = attn_keep_mask(B, H, N, rng, site, p, pr.device, bh0).float() / (1.0 - p)
    else:
        m = torch.ones_like(pr)
    pd = pr * m
    dv = bf16(pd).float().transpose(-1, -2) @ dof
    dpd = dof @ v.transpose(-1, -2)
    dp = dpd * m
    delta = (dof * of).sum(-1, keepdim=True)
    ds = pr * (dp - delta)
    dq = (bf16(ds).float() @ k) * scale
    dk = (bf16(ds).float().transpose(-1, -2) @ q) * scale
    d = torch.stack((dq, dk, dv), dim=0)  # [3,B,H,N,hd]
    return bf16(d.permute(1, 3, 0, 2, 4).reshape(B * N, 3 * H * hd))


def embed_patch_grad(g, rng, site: int, p: float):
    """The patch-row gradient of :func:`embed_bwd` alone: token rows 1..N-1 of ``g``
    ([B, N, D]) with the embedding dropout, bf16, [B*(N-1), D]."""
    B, N, D = g.shape
    return bf16(_dropout(g.float(), rng, site, p)[:, 1:, :].reshape(B * (N - 1), D))


def embed_bwd(g, t, rng, site: int, p: float, dcls, dpos, dtemb):
    """Grads of cls/pos/time embeddings (+=) and the patch-row grad (bf16) for the conv wgrad."""
    B, N, D = g.shape
    gm = _dropout(g.float(), rng, site, p)
    dcls.view(-1).add_(gm[:, 0, :].sum(0))
    dpos.view(N, D).add_(gm.sum(0))
    dtemb.index_add_(0, t, gm.sum(1))
    return bf16(gm[:, 1:, :].reshape(B * (N - 1), D))


# ----------------------------------------------------------------------------- diffusion / data ops
def ddim_coeffs(total_steps: int, t: int, k: int):
    """(sqrt(a_t), sqrt(1-a_t), sqrt(a_{t-k}), sqrt(1-a_{t-k})) for the sqrt schedule.

    a(t) = 1 - sqrt((t+1)/T) + 1e-5 for the current step (`ViT.py:232`) and
    a(t-k) = 1 - sqrt((t+1-k)/T) (no epsilon, `ViT.py:231`).
    """
    a_t = 1.0 - math.sqrt((t + 1) / total_steps) + 1e-5
    a_tk = 1.0 - math.sqrt((t + 1 - k) / total_steps)
    if a_tk <= 0.0:
        raise ValueError(f"DDIM step jump k={k} must divide total_steps={total_steps}")
    return math.sqrt(a_t), math.sqrt(1.0 - a_t), math.sqrt(a_tk), math.sqrt(1.0 - a_tk)


def ddim_step(x_t, x0_raw, coef):
    """Fused clamp + eps-hat + DDIM update (fp32); returns (x_{t-k}, clamped x0)."""
    sa, s1a, sak, s1ak = coef
    x0 = torch.clamp(x0_raw, -1.0, 1.0)
    eps = (x_t - sa * x0) / s1a
    return sak * x0 + s1ak * eps, x0


def pixelate(img, factor: int):
    """NEAREST down to floor(W/f) then NEAREST up (`diffusion_loader.py:79-83`)."""
    H, W = img.shape[-2:]
    ts = max(int(math.floor(W / factor)), 1)
    small = F.interpolate(img, size=(ts, ts), mode="nearest")
    return F.interpolate(small, size=(H, W), mode="nearest")


def img_to_tokgrad_op(dimg, N: int, patch: int):
    return img_to_tokgrad(dimg, N, patch)


def q_sample(x0, t, eps, total_steps: int):
    """sqrt(a)*x0 + sqrt(1-a)*eps with a = 1 - sqrt((t+1)/T) (`diffusion_loader.py:50-54`)."""
    a = 1.0 - torch.sqrt((t.double() + 1.0) / total_steps)
    a = a.float().view(-1, 1, 1, 1)
    return torch.sqrt(a) * x0 + torch.sqrt(1.0 - a) * eps
