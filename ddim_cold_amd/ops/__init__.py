"""Fused-op layer: one Python entry point per HIP kernel op.

GPU tensors go to ``torch.ops.ddim_cold.<op>`` (hand-written gfx950 kernels in
``csrc/``); CPU tensors go to the bit-compatible PyTorch reference in
:mod:`.reference`.  On a GPU the native path is mandatory (see
:mod:`._ext`): a missing extension raises instead of silently running eager
PyTorch.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _ext
from . import reference as ref
from ._ext import force_reference

__all__ = [
    "native_available", "patch_embed_fwd", "layernorm_fwd", "qkv_fwd", "attn_fwd", "attn_keep_buffer",
    "linear_residual_fwd", "linear_gelu_fwd", "head_fwd", "smooth_l1_fwd_bwd", "img_to_tokgrad",
    "linear_dgrad", "linear_dgrad_gelu", "linear_wgrad", "layernorm_bwd", "attn_bwd", "embed_bwd",
    "sqnorm", "adamw_step", "advance_counters", "ddim_step", "ddim_step_", "randn_", "q_sample",
    "pixelate_pair", "cold_batch", "gauss_batch", "head_step_rows_",
    "image_to_rows", "rows_to_image", "embed_weight_rows", "patch_embed_cold_fwd", "ln_fold_",
]


def native_available() -> bool:
    return _ext.available()


def _hip(t: torch.Tensor) -> bool:
    return _ext.require_for(t)


def _ops():
    return torch.ops.ddim_cold


# ----------------------------------------------------------------------------- forward
def patch_embed_fwd(img, t, w_pe, b_pe, cls, pos, temb, rng, site: int, p: float, patch: int, ln_st=None,
                    xb_out=None, patches_in=None):
    """Tokens + bf16 patches.  LayerNorm fold: ``ln_st`` ([B*N, D/32, 2]) gets the
    tokens' row statistics ({sum, sum^2} per 32-column slot); ``xb_out`` their
    bf16 copy (the A operand of the first QKV GEMM).  ``patches_in``: the bf16
    patch rows of ``img`` already exist (a sampler step's :func:`head_step_` wrote
    them) -- on a GPU the patchify launch is skipped (the GEMM writes the cls rows)."""
    if _hip(img):
        return _ops().patch_embed_fwd(img, t, w_pe, b_pe, cls, pos, temb, rng, site, float(p), patch, ln_st, xb_out,
                                      patches_in)
    return ref.patch_embed_fwd(img, t, w_pe, b_pe, cls, pos, temb, rng, site, p, patch, ln_st, xb_out)


def patch_embed_cold_fwd(cold, img, t, w_pe, b_pe, cls, pos, temb, rng, site: int, p: float, patch: int,
                         ln_st=None, xb_out=None, target_rows: bool = False):
    """:func:`cold_batch` fused into :func:`patch_embed_fwd` (one launch fewer per
    training step): ``cold = (pool, data_site, max_t, draw_idx, target_x0, target,
    idx, write_xt)``; the patch rows are pixelated straight from the pool, ``target``,
    ``t`` and (if ``draw_idx``) ``idx`` are written, ``img`` (x_t) only if ``write_xt``.
    Same values as ``cold_batch`` then ``patch_embed_fwd``.  Two optional trailing
    entries ``(gauss_T, noise_site)`` with ``gauss_T > 0`` select the Gaussian DDIM
    batch instead (same values as :func:`gauss_batch` then ``patch_embed_fwd``).
    ``target_rows``: the target is written as patch rows in the head's output column
    order (:func:`image_to_rows`) into the same buffer, for :func:`head_loss` with
    ``target_rows``.  An 11th entry ``idx_step = (ctr, off)`` (or None): ``idx`` is a
    stepped table read at row ``ctr[0] % rows`` (see :func:`stepped_idx`)."""
    pool, dsite, max_t, draw, tx0, target, idx, write_xt = cold[:8]
    gT, nsite = (int(cold[8]), int(cold[9])) if len(cold) > 8 else (0, 0)
    step = cold[10] if len(cold) > 10 else None
    if _hip(img):
        ctr, off = step if step is not None else (None, 0)
        return _ops().patch_embed_cold_fwd(pool, int(dsite), int(max_t), bool(draw), bool(tx0), img, target, t, idx,
                                           bool(write_xt), w_pe, b_pe, cls, pos, temb, rng, site, float(p), patch,
                                           ln_st, xb_out, gT, nsite, bool(target_rows), ctr, int(off))
    if gT > 0:
        gauss_batch(pool, rng, dsite, nsite, gT, img, target, t, idx, draw, idx_step=step)
    else:
        cold_batch(pool, rng, dsite, img, target, t, idx, max_t, draw, idx_step=step)
        if tx0:
            torch.index_select(pool, 0, stepped_idx(idx, step, img.shape[0]), out=target)
    if target_rows:
        target.copy_(image_to_rows(target.clone(), patch).reshape(target.shape))
    return patch_embed_fwd(img, t, w_pe, b_pe, cls, pos, temb, rng, site, p, patch, ln_st, xb_out)


def layernorm_fwd(x, gamma, beta, eps: float = 1e-5):
    if _hip(x):
        return _ops().layernorm_fwd(x, gamma, beta, float(eps))
    return ref.layernorm_fwd(x, gamma, beta, eps)


def linear_fwd(a, w, b=None, out_fp32: bool = False, fold=None):
    """Plain ``a @ w.T + b`` on the MFMA GEMM (bf16 or fp32 output).  ``fold =
    (ln_st, ln_c, eps)``: LayerNorm folded in (``a`` = raw rows, ``w``/``b`` folded)."""
    st, c, eps = fold if fold is not None else (None, None, 1e-5)
    if _hip(a):
        return _ops().linear_fwd(a, w, b, bool(out_fp32), st, c, float(eps))
    return ref.linear_fwd(a, w, b, out_fp32, st, c, eps)


def _fold_args(fold):
    """``fold = (ln_st, ln_c, eps[, mean_out, rstd_out])`` -> op keyword tuple."""
    if fold is None:
        return None, None, 1e-5, None, None
    st, c, eps = fold[:3]
    mean, rstd = (fold[3], fold[4]) if len(fold) > 3 else (None, None)
    return st, c, float(eps), mean, rstd


def qkv_fwd(a, w, b, B: int, N: int, H: int, fold=None):
    """QKV projection, head-major [3,B,H,N,hd].  ``fold = (ln_st, ln_c, eps, mean_out,
    rstd_out)``: the preceding LayerNorm folded in (``a`` = bf16 residual rows,
    ``w``/``b`` from :func:`ln_fold_`); mean/rstd of the rows written for the backward."""
    st, c, eps, mean, rstd = _fold_args(fold)
    if _hip(a):
        return _ops().qkv_fwd(a, w, b, B, N, H, st, c, eps, mean, rstd)
    return ref.qkv_fwd(a, w, b, B, N, H, st, c, eps, mean, rstd)


class gemm_tile:
    """Context manager forcing the GEMM tile config of every launch inside it
    (csrc/gemm.hip: 0 = 32x64, 1 = 64x64, 2 = 128x64, 3 = 128x128 with 4 waves;
    4 = 256x128, 5 = 128x128 with 8 waves; -1 = automatic).  Tests and
    micro-benchmarks; the automatic choice is the production path."""

    def __init__(self, cfg: int):
        self.cfg = int(cfg)
        self.prev = -1

    def __enter__(self):
        _ext.load(raise_on_error=True)
        self.prev = int(_ops().gemm_tile_override(self.cfg))
        return self

    def __exit__(self, *exc):
        _ops().gemm_tile_override(self.prev)
        return False


def attn_keep_buffer(qkv, p: float):
    """int32 buffer for the attention-dropout keep flags the forward stores for its
    backward (short sequences: one word per lane; long ones: one 64-bit word per
    query and 64-key tile), so the backward reads masks instead of re-hashing them;
    None when there is nothing to store (p = 0, CPU, or the one long-sequence
    forward that keeps no words: 320 < N < 384 with fewer than 192 heads)."""
    if p <= 0 or not _hip(qkv):
        return None
    _, B, H, N, hd = qkv.shape
    n = int(_ops().attn_keep_words(B, H, N, hd))
    return torch.empty(n, dtype=torch.int32, device=qkv.device) if n > 0 else None


def attn_fwd(qkv, scale: float, rng, site: int, p: float, keep_out=None):
    """``keep_out`` (:func:`attn_keep_buffer`): also store the dropout keep flags."""
    if _hip(qkv):
        return _ops().attn_fwd(qkv, float(scale), rng, site, float(p), keep_out)
    return ref.attn_fwd(qkv, scale, rng, site, p)


def linear_residual_fwd(a, w, b, x, N: int, rng, site_drop: int, p_drop: float, site_dp: int, p_dp: float,
                        st_out=None, xb_out=None):
    """x + DropPath(Dropout(a w^T + b)).  LayerNorm fold producer: ``st_out`` ([M, D/32, 2])
    gets the new rows' {sum, sum^2} per 32-column slot, ``xb_out`` their bf16 copy."""
    if _hip(a):
        return _ops().linear_residual_fwd(a, w, b, x, N, rng, site_drop, float(p_drop), site_dp, float(p_dp),
                                          st_out, xb_out)
    return ref.linear_residual_fwd(a, w, b, x, N, rng, site_drop, p_drop, site_dp, p_dp, st_out, xb_out)


def linear_gelu_fwd(a, w, b, rng, site: int, p: float, fold=None):
    st, c, eps, mean, rstd = _fold_args(fold)
    if _hip(a):
        return _ops().linear_gelu_fwd(a, w, b, rng, site, float(p), st, c, eps, mean, rstd)
    return ref.linear_gelu_fwd(a, w, b, rng, site, p, st, c, eps, mean, rstd)


def _ddim_coef(coef, x):
    """4 DDIM coefficients as python floats (one row) or [B,1,1,1] tensors (one row per sample)."""
    if coef.dim() == 2:
        return [coef[:, i].reshape(-1, 1, 1, 1).to(x.dtype) for i in range(4)]
    return [float(c) for c in coef.tolist()[:4]]


def head_step_(a, w, b, x, x0_out, coef, patch: int, mode: int, fold=None, patches_out=None):
    """Head GEMM + sampler step in its epilogue (in place on ``x``): mode 1 = clamp +
    DDIM update (``x0_out`` gets the clamped x0-hat; ``coef`` a device row of
    ``ddim_coefficients``), mode 2 = clamp only (cold sampler), mode 4 = mode 1 with
    one coefficient row per sample (``coef`` [B, 4]; img2img: the row {0, 1, 0, 1}
    leaves a sample that has not reached its start step unchanged).  ``patches_out``
    (GPU): also the new ``x`` as bf16 patch rows, for the next step's
    :func:`patch_embed_fwd` (``patches_in``)."""
    st, c, eps, _, _ = _fold_args(fold)
    if _hip(a):
        return _ops().head_step_(a, w, b, x, x0_out, coef, patch, mode, st, c, eps, patches_out)
    B, C, H, W = x.shape
    x0_raw = ref.head_fwd(a, w, b, B, C, H, W, patch, st, c, eps)
    if mode == 2:
        x.copy_(torch.clamp(x0_raw, -1.0, 1.0))
        return
    xn, x0 = ref.ddim_step(x, x0_raw, _ddim_coef(coef, x))
    x.copy_(xn)
    x0_out.copy_(x0)


def image_to_rows(x, patch: int):
    """[B,C,H,W] -> [B*P, C*p*p] patch rows in the head's output column order
    ((a*p + b)*C + c for pixel (a, b) of the patch, channel c; ViT.py:214-217 unpatchify)."""
    B, C, H, W = x.shape
    p = patch
    return x.reshape(B, C, H // p, p, W // p, p).permute(0, 2, 4, 3, 5, 1).reshape(B * (H // p) * (W // p), p * p * C)


def rows_to_image(xr, B: int, C: int, H: int, W: int, patch: int):
    """Inverse of :func:`image_to_rows`."""
    p = patch
    return xr.reshape(B, H // p, W // p, p, p, C).permute(0, 5, 1, 3, 2, 4).reshape(B, C, H, W)


def embed_weight_rows(w_pe, C: int, patch: int):
    """Patch-embedding weight [D, C*p*p] (conv order c, a, b) with its columns permuted
    to the head's output order, so bf16 patch rows in that order (:func:`head_step_rows_`
    ``patches_out``) feed :func:`patch_embed_fwd` ``patches_in`` directly."""
    D = w_pe.shape[0]
    return w_pe.reshape(D, C, patch, patch).permute(0, 2, 3, 1).reshape(D, C * patch * patch)


def head_step_rows_(a, w, b, x, x0_out, coef, batch: int, mode: int, fold=None, patches_out=None):
    """:func:`head_step_` on patch rows (``x``/``x0_out``/``patches_out`` [B*P, F] in the
    head's output column order, :func:`image_to_rows`): every epilogue access is a
    contiguous vector instead of a scattered pixel.  Same math per element."""
    st, c, eps, _, _ = _fold_args(fold)
    if _hip(a):
        return _ops().head_step_rows_(a, w, b, x, x0_out, coef, int(batch), int(mode), st, c, eps, patches_out)
    F = w.shape[0]
    NP = x.shape[0] // batch
    y = ref._lin(a, w, b, st, c, eps)
    y = y.reshape(batch, NP + 1, F)[:, 1:].reshape(batch * NP, F)
    x0 = torch.clamp(y, -1.0, 1.0)
    if mode == 2:
        x.copy_(x0)
    else:
        cf = coef.reshape(-1, 4).float()
        cf = cf.repeat_interleave(NP, 0) if cf.shape[0] == batch and mode == 4 else cf[:1].expand(x.shape[0], 4)
        eps_hat = (x - cf[:, 0:1] * x0) / cf[:, 1:2]
        x.copy_(cf[:, 2:3] * x0 + cf[:, 3:4] * eps_hat)
        x0_out.copy_(x0)
    if patches_out is not None:
        patches_out.copy_(x)


def head_fwd(a, w, b, B: int, C: int, H: int, W: int, patch: int, fold=None):
    st, c, eps, mean, rstd = _fold_args(fold)
    if _hip(a):
        return _ops().head_fwd(a, w, b, B, C, H, W, patch, st, c, eps, mean, rstd)
    return ref.head_fwd(a, w, b, B, C, H, W, patch, st, c, eps, mean, rstd)


def head_loss(a, w, b, target, patch: int, beta: float = 1.0, fold=None, target_rows: bool = False):
    """Head GEMM + mean smooth-L1 vs ``target`` + its gradient in the token layout, in
    one launch: ``(loss_parts, dtok)`` -- the loss is ``loss_parts.sum()`` (finished by
    the step tail of :func:`ln_fold_`); the predicted image is never materialised.
    ``target_rows``: the [B, C, H, W]-shaped ``target`` buffer holds patch rows in the
    head's output order (:func:`image_to_rows`; vector epilogue on a GPU)."""
    st, c, eps, mean, rstd = _fold_args(fold)
    if _hip(a):
        return _ops().head_loss(a, w, b, target, patch, float(beta), st, c, eps, mean, rstd, bool(target_rows))
    B, C, H, W = target.shape
    if target_rows:
        target = rows_to_image(target.reshape(-1, C * patch * patch), B, C, H, W, patch)
    out = ref.head_fwd(a, w, b, B, C, H, W, patch, st, c, eps, mean, rstd)
    N = a.shape[0] // B
    loss, dtok = ref.smooth_l1_fwd_bwd(out, target, N, patch, beta)
    return loss.reshape(1), dtok


def smooth_l1_fwd_bwd(pred, target, N: int, patch: int, beta: float = 1.0, loss_last=None, loss_ema=None,
                      ema_decay: float = 0.99, finish: bool = True):
    """Mean smooth-L1 loss and its token-layout gradient; optionally also writes
    ``loss_last`` and updates ``loss_ema`` (decay) in the same launch.  ``finish=False``
    returns the loss as per-block partials (summed later by the step tail of
    :func:`ln_fold_`) instead of launching the finishing reduction."""
    if _hip(pred):
        return _ops().smooth_l1_fwd_bwd(pred, target, N, patch, float(beta), loss_last, loss_ema, float(ema_decay),
                                        bool(finish))
    loss, dtok = ref.smooth_l1_fwd_bwd(pred, target, N, patch, beta)
    if not finish:
        return loss.reshape(1), dtok
    if loss_last is not None:
        loss_last.copy_(loss.reshape(loss_last.shape))
    if loss_ema is not None:
        loss_ema.mul_(ema_decay).add_(loss.reshape(loss_ema.shape), alpha=1.0 - ema_decay)
    return loss, dtok


def img_to_tokgrad(dimg, N: int, patch: int):
    if _hip(dimg):
        return _ops().img_to_tokgrad(dimg.contiguous(), N, patch)
    return ref.img_to_tokgrad(dimg, N, patch)


# ----------------------------------------------------------------------------- backward
def linear_dgrad(dy, w, out_fp32: bool, splits: int = 1):
    """``dy @ W``.  ``splits`` > 1: ``[splits, M, K]`` partial products (fp32 or
    bf16) over slices of the reduction dim, written without atomics or zeroing;
    :func:`layernorm_bwd` sums them (in fp32) as it loads ``dy``."""
    if _hip(dy):
        return _ops().linear_dgrad(dy, w, bool(out_fp32), int(splits))
    return ref.linear_dgrad(dy, w, out_fp32, splits)


def linear_dgrad_gelu(dy, w, u, rng, site: int, p: float, wt=None):
    """``(dy @ W) * gelu'(u)`` with the dropout mask of ``site``; ``wt`` (= W^T, bf16
    [in][out]): the product on the k-contiguous operand path."""
    if _hip(dy):
        if wt is not None:
            return _ops().linear_dgrad_gelu_t(dy, wt, u, rng, site, float(p))
        return _ops().linear_dgrad_gelu(dy, w, u, rng, site, float(p))
    return ref.linear_dgrad_gelu(dy, w, u, rng, site, p)


def linear_wgrad(dy, x, dw, db: Optional[torch.Tensor]):
    if _hip(dy):
        return _ops().linear_wgrad(dy, x, dw, db)
    return ref.linear_wgrad(dy, x, dw, db)


def wire_pack(src, dst):
    """fp32 -> bf16 (round to nearest even) into ``dst`` (gradient wire format)."""
    if _hip(src):
        return _ops().wire_pack(src, dst)
    dst.copy_(src)


def wire_unpack(src, dst):
    """bf16 -> fp32 into ``dst``."""
    if _hip(src):
        return _ops().wire_unpack(src, dst)
    dst.copy_(src)


def wgrad_embed_slots(B: int, N: int, D: int, owners: int, n_ln: int, ln_C: int, wide: bool) -> int:
    """Grad-norm partial slots (= extra workgroups) the embedding parts of
    :func:`linear_wgrad_multi` take (``wide``: the 512-thread tiles of >= 16,384-token
    reductions)."""
    nt = 512 if wide else 256
    return -(-(N * D) // nt) + owners * -(-D // 16) + (n_ln * -(-ln_C // 16) if n_ln else 0)


def linear_wgrad_multi(jobs, store: bool = False, sq=None, embed=None):
    """Every ``(dy, x, dw, db)`` weight-gradient job of a step (<= 32) in ONE launch
    (csrc/gemm.hip ``gemm_wgrad_multi_kernel``; unsplit, deterministic).  ``store``:
    the targets are zero (``dW = dy^T x`` written, not added: no read of dW).

    ``sq = (parts, arena, lazy)``: the launch is the last writer of the gradient
    ``arena`` (every dw / db a view of it), so it also writes the grad-norm partials
    :func:`sqnorm` would (same buffer layout, scale 1): each output tile the sum of
    squares of its final values, extra workgroups the arena ranges outside every
    target and outside ``lazy`` = (lo, hi).  Replaces the separate sqnorm pass.

    ``embed = (g, t, rng, site, p, dcls, dpos, dtemb, owners, ln)``: the cls / pos /
    time-embedding gradients of :func:`embed_bwd` (parts A, B; ``g`` the embedding
    output gradient [B, N, D], ``owners`` >= the distinct timesteps a batch can hold)
    and, with ``ln = (ws, dst_ptrs, offs, C, R, store)``, the LayerNorm slot finalize
    ride in the same launch as extra workgroups (each writing the grad-norm partials of
    its outputs); the patch-row gradient comes from the last LayerNorm backward
    (:func:`layernorm_bwd` ``gp_out``).  Deterministic."""
    if not jobs:
        return
    if _hip(jobs[0][0]):  # (more than 32 jobs: consecutive launches of <= 32)
        dys, xs, dws, dbs = (list(z) for z in zip(*jobs))
        parts, arena, (lo, hi) = (None, None, (0, 0)) if sq is None else \
            (sq[0], sq[1], sq[2] if sq[2] is not None else (0, 0))
        if embed is None:
            _ops().linear_wgrad_multi(dys, xs, dws, dbs, bool(store), parts, arena, int(lo), int(hi))
            return
        g, t, rng, site, p, dcls, dpos, dtemb, owners, ln = embed
        lw, lp, loffs, lC, lR, lst = ln if ln is not None else (None, None, [], 0, 0, False)
        _ops().linear_wgrad_multi(dys, xs, dws, dbs, bool(store), parts, arena, int(lo), int(hi), g, t, rng,
                                  int(site), float(p), dcls, dpos, dtemb, int(owners), lw, lp,
                                  [int(o) for o in loffs], int(lC), int(lR), bool(lst))
        return
    for dy, x, dw, db in jobs:
        if store:
            dw.zero_()
            if db is not None:
                db.zero_()
        ref.linear_wgrad(dy, x, dw, db)
    if embed is not None:
        g, t, rng, site, p, dcls, dpos, dtemb, owners, ln = embed
        ref.embed_bwd(g, t, rng, site, p, dcls, dpos, dtemb)
        if ln is not None:
            raise ValueError("the LayerNorm finalize in the weight-gradient launch needs the HIP extension")
    if sq is not None:
        parts, arena, lazy = sq
        sqnorm(arena, parts, 1.0, lazy=lazy)


def transpose_bf16_(srcs, dsts):
    """``dsts[i] = srcs[i].T`` for bf16 matrices (one launch per 96; csrc/transpose.hip):
    the transposed weight shadows the input-gradient GEMMs read k-contiguous."""
    if srcs and _hip(srcs[0]):
        _ops().transpose_bf16_(list(srcs), list(dsts))
        return
    for s_, d_ in zip(srcs, dsts):
        d_.copy_(s_.t())


def ln_ws_rows(M: int) -> int:
    """Rows ([rows, 2D] floats) of the dgamma||dbeta workspace :func:`layernorm_bwd`
    takes for ``M`` rows: one slot per backward workgroup (csrc/layernorm.hip: 8 rows per
    workgroup, at most 512 workgroups), each overwritten by its workgroup, summed in slot
    order by :func:`replica_reduce_` (deterministic, no atomics).  The loaded extension's
    own count when there is one (one source of truth; A/B runs load other builds)."""
    if native_available():
        return int(_ops().ln_ws_rows(int(M)))
    return max(1, min(-(-M // 8), 512))


def layernorm_bwd(dy, x, mean, rstd, gamma, g_res, dgamma, dbeta, N: int, rng, site_drop: int, p_drop: float,
                  site_dp: int, p_dp: float, emit_gy: bool, ws: Optional[torch.Tensor] = None, beta=None,
                  y_out=None, gp_out=None, site_emb: int = 0, p_emb: float = 0.0):
    """LayerNorm backward.  With ``ws`` ([ln_ws_rows(M), 2D]) the dgamma||dbeta
    partials stay in the workspace slots (finalise later with :func:`replica_reduce_`;
    deterministic, no atomics); otherwise they are added into dgamma / dbeta.
    ``y_out`` (with ``beta``): also write the LayerNorm output (bf16) — the
    forward folded the LayerNorm into the next GEMM and never stored it.
    ``gp_out`` ([B*(N-1), D] bf16; the last LayerNorm of the backward): also write the
    patch-embedding input gradient, g_out's token rows 1..N-1 with the embedding
    dropout (``site_emb``, ``p_emb``) -- what :func:`embed_bwd` returns."""
    if _hip(x):
        g_out, gy = _ops().layernorm_bwd(dy, x, mean, rstd, gamma, g_res, dgamma, dbeta, N, rng, site_drop,
                                         float(p_drop), site_dp, float(p_dp), bool(emit_gy), ws, beta, y_out,
                                         gp_out, int(site_emb), float(p_emb))
        return g_out, (gy if emit_gy else None)
    if ws is not None:
        D = x.shape[-1]
        dgamma, dbeta = ws[0, :D], ws[0, D:]
    if y_out is not None:
        ref.layernorm_out_(x, mean, rstd, gamma, beta, y_out)
    g_out, gy = ref.layernorm_bwd(dy, x, mean, rstd, gamma, g_res, dgamma, dbeta, N, rng, site_drop, p_drop,
                                  site_dp, p_dp, emit_gy)
    if gp_out is not None:
        gp_out.copy_(ref.embed_patch_grad(g_out.view(-1, N, x.shape[-1]), rng, site_emb, p_emb))
    return g_out, gy


def ln_fold_(ws, gammas, betas, biases, wfs, cs, bfs, tail=None):
    """LayerNorm fold weights for GEMMs that consume a LayerNorm (one launch on GPU):
    ``wf = bf16(gamma o W)``, ``c = rowsum(wf)``, ``bf = b + W beta``.

    ``tail = (loss_parts, loss_last, loss_ema, ema_decay, step, rng, sq)``: the
    training step's tail rides in the same launch -- loss from the smooth-L1
    partials (``loss_last``, EMA) and the counter advance of
    :func:`advance_counters` (optimizer step only if the grad norm ``sq`` is finite)."""
    if not ws:
        return
    if _hip(ws[0]):
        t = tail if tail is not None else (None, None, None, 0.99, None, None, None)
        return _ops().ln_fold_(list(ws), list(gammas), list(betas), list(biases), list(wfs), list(cs), list(bfs),
                               t[0], t[1], t[2], float(t[3]), t[4], t[5], t[6])
    for w, g, be, b, wf, c, bf in zip(ws, gammas, betas, biases, wfs, cs, bfs):
        ref.ln_fold(w, g, be, b, wf, c, bf)
    if tail is not None:
        parts, loss_last, loss_ema, decay, step, rng, sq = tail
        loss = parts.float().sum().reshape(1)
        if loss_last is not None:
            loss_last.copy_(loss.reshape(loss_last.shape))
        if loss_ema is not None:
            loss_ema.mul_(decay).add_(loss.reshape(loss_ema.shape), alpha=1.0 - decay)
        advance_counters(step, rng, sq)


def replica_reduce_(ws, dst_ptrs, C: int, R: int, dsts=None):
    """dst[g] += ws[g, :R].sum(0) (rows in order) for G LayerNorm workspaces
    ([G, rows, C]; ``R`` = :func:`ln_ws_rows` of the backward's row count).

    ``dst_ptrs`` is a device int64 tensor of destination addresses (GPU); the
    CPU path takes the destination tensors in ``dsts`` instead (and re-zeroes the
    rows: its LayerNorm backward accumulates into row 0)."""
    if _hip(ws):
        return _ops().replica_reduce_(ws, dst_ptrs, C, int(R))
    for g, d in enumerate(dsts):
        d.add_(ws[g, :R].sum(0))
    ws[:, :R].zero_()


def attn_bwd(do, qkv, o, lse, scale: float, rng, site: int, p: float, keep=None):
    """``keep``: the keep flags :func:`attn_fwd` stored (same masks as re-hashing)."""
    if _hip(qkv):
        return _ops().attn_bwd(do, qkv, o, lse, float(scale), rng, site, float(p), keep)
    return ref.attn_bwd(do, qkv, o, lse, scale, rng, site, p)


def embed_bwd(g, t, rng, site: int, p: float, dcls, dpos, dtemb, ln_final=None):
    """``ln_final = (ws, dst_ptrs, C, R[, store])``: the LayerNorm finalize
    (:func:`replica_reduce_`) rides in the same launch (GPU only); ``store``: the
    destinations get the sum instead of having it added.  Deterministic: no fp32
    atomics (the time-embedding rows are summed per distinct timestep)."""
    if _hip(g):
        ws, ptrs, C, R = ln_final[:4] if ln_final is not None else (None, None, 0, 0)
        store = bool(ln_final[4]) if ln_final is not None and len(ln_final) > 4 else False
        return _ops().embed_bwd(g, t, rng, site, float(p), dcls, dpos, dtemb, ws, ptrs, int(C), store, int(R))
    if ln_final is not None:
        raise ValueError("ln_final needs the HIP extension (use replica_reduce_ on CPU)")
    return ref.embed_bwd(g, t, rng, site, p, dcls, dpos, dtemb)


# ----------------------------------------------------------------------------- optimizer
SQ_PARTS = 1024  # csrc/kernels.h


def sq_parts_size(n_tiles: int) -> int:
    """Grad-norm partial buffer size (floats) for a fused weight-gradient launch of
    ``n_tiles`` 64x64 tiles: room for the tiles, up to 64 tail workgroups, >= SQ_PARTS,
    a multiple of 256 (what every consumer kernel accepts)."""
    n = max(SQ_PARTS, n_tiles + 64)
    return (n + 255) // 256 * 256


def sqnorm(g, out, scale: float = 1.0, lazy=None):
    """Per-block partial sums of (g*scale)^2 into ``out`` (>= SQ_PARTS floats, a multiple
    of 256, fully overwritten).
    ``lazy`` = (lo, hi): an arena range whose gradient is identically zero (skipped)."""
    lo, hi = lazy if lazy is not None else (0, 0)
    if _hip(g):
        return _ops().sqnorm(g, out, float(scale), int(lo), int(hi))
    out.zero_()
    out[0] = (g.float() * scale).pow(2).sum()


def adamw_step(p, g, m, v, pbf, sq, step, hyper, grad_scale: float = 1.0, zero_hi: Optional[int] = None,
               lazy=None, lazy_decay=None):
    """Fused AdamW over a flat arena (see csrc/optim.hip for the exact math).
    ``zero_hi``: zero the gradients only below this element (the producers of the
    rest overwrite them next step); default: all.  ``lazy`` = (lo, hi) with
    ``lazy_decay`` (fp32 [1]): parameters whose gradient and moments are identically
    zero; they are not touched, their weight decay (1 - lr*wd per step) accumulates
    into ``lazy_decay`` for ``TrainEngine.materialize_lazy``."""
    lo, hi = lazy if lazy is not None and lazy_decay is not None else (0, 0)
    if _hip(p):
        return _ops().adamw_step(p, g, m, v, pbf, sq, step, hyper, float(grad_scale),
                                 -1 if zero_hi is None else int(zero_hi), int(lo), int(hi), lazy_decay)
    import math
    sqv = float(sq.sum())
    base_lr, b1, b2, eps, wd, max_norm, tmax, eta_min = (float(x) for x in hyper.tolist()[:8])
    coef = grad_scale
    if max_norm > 0:
        coef *= min(1.0, max_norm / (math.sqrt(sqv) + 1e-6)) if math.isfinite(sqv) else 1.0
    gi = g * coef
    g[: (g.numel() if zero_hi is None else zero_hi)].zero_()
    if not math.isfinite(sqv):
        return
    t = int(step[0]) + 1
    bc1, bc2 = 1 - b1 ** t, 1 - b2 ** t
    lr = base_lr
    if tmax > 0:
        lr = eta_min + (base_lr - eta_min) * 0.5 * (1 + math.cos(math.pi * int(step[1]) / tmax))
    if hi > lo:  # the lazy range: untouched, its decay accumulated (same as the kernel)
        keep = (p[lo:hi].clone(), m[lo:hi].clone(), v[lo:hi].clone())
        lazy_decay.mul_(1 - lr * wd)
    p.mul_(1 - lr * wd)
    m.mul_(b1).add_(gi, alpha=1 - b1)
    v.mul_(b2).addcmul_(gi, gi, value=1 - b2)
    p.addcdiv_(m, v.sqrt() / math.sqrt(bc2) + eps, value=-lr / bc1)
    if hi > lo:
        p[lo:hi], m[lo:hi], v[lo:hi] = keep
    if pbf is not None:
        pbf.copy_(p.to(torch.bfloat16))


def advance_counters(step, rng, sq=None):
    if _hip(step):
        return _ops().advance_counters(step, rng, sq)
    import math
    if sq is None or math.isfinite(float(sq.sum())):
        step[0] += 1
    step[1] += 1
    rng[1] += 1


# ----------------------------------------------------------------------------- diffusion / data
def ddim_step(x_t, x0_raw, coef):
    if _hip(x_t):
        return _ops().ddim_step(x_t, x0_raw, coef)
    return ref.ddim_step(x_t, x0_raw, [float(c) for c in coef.tolist()[:4]])


def ddim_step_(x, x0_raw, x0_out, coef):
    """In-place DDIM step; ``coef`` one row of 4 (GPU kernel) or [B, 4] per sample (torch ops)."""
    if _hip(x) and coef.dim() == 1:
        return _ops().ddim_step_(x, x0_raw, x0_out, coef)
    xn, x0 = ref.ddim_step(x, x0_raw, _ddim_coef(coef, x))
    x.copy_(xn)
    x0_out.copy_(x0)


def randn_(out, rng, site: int):
    if _hip(out):
        return _ops().randn_(out, rng, site)
    salt = ref.site_salt(rng, site)
    n = out.numel()
    pairs = (n + 1) // 2
    i = torch.arange(pairs, dtype=torch.int64)
    ha = ref.mix32(ref._mul32((2 * i) & ref.MASK32, ref.GOLDEN) ^ salt)
    hb = ref.mix32(ref._mul32((2 * i + 1) & ref.MASK32, ref.GOLDEN) ^ salt)
    a = ((ha >> 8).double() + 0.5) / 16777216.0
    b = ((hb >> 8).double() + 0.5) / 16777216.0
    r = torch.sqrt(-2.0 * torch.log(a))
    z = torch.stack((r * torch.cos(2 * torch.pi * b), r * torch.sin(2 * torch.pi * b)), dim=1).reshape(-1)[:n]
    out.copy_(z.float().view(out.shape))


def q_sample(x0, t, eps, total_steps: int):
    if _hip(x0):
        return _ops().q_sample(x0, t, eps, total_steps)
    return ref.q_sample(x0, t, eps, total_steps)


def pixelate_pair(img, idx, t, B: int):
    if _hip(img):
        return _ops().pixelate_pair(img, idx, t, B)
    src = img if idx is None else img[idx]
    xt = torch.stack([ref.pixelate(src[i:i + 1], 2 ** int(t[i]))[0] for i in range(B)])
    xtm1 = torch.stack([ref.pixelate(src[i:i + 1], 2 ** (int(t[i]) - 1))[0] for i in range(B)])
    return xt, xtm1


def stepped_idx(idx, idx_step, B: int):
    """The [B] pool indices a batch source reads: ``idx`` itself, or with ``idx_step =
    (ctr, off)`` row ``ctr[0] % rows`` of the stepped table ``idx`` ([rows, ...]),
    elements ``off .. off+B`` (the trainer's epoch table indexed by the device step
    counter, so a K-step graph needs no host copy per step)."""
    if idx_step is None:
        return idx
    ctr, off = idx_step
    r = torch.remainder(ctr.reshape(-1)[:1], idx.shape[0])  # device ops: graph-capturable, no host sync
    return idx.reshape(idx.shape[0], -1).index_select(0, r)[0, int(off):int(off) + B]


def gauss_batch(pool, rng, site: int, noise_site: int, total_steps: int, x_t, x0, t, idx, draw_idx: bool = True,
                idx_step=None):
    """Gaussian DDIM batch on device in one launch (diffusion_loader.py:24-58): pool
    index (unless ``draw_idx`` is False: ``idx`` holds them; ``idx_step``: see
    :func:`stepped_idx`) and t ~ U{0..T-1} from the ``site`` hash, eps =
    :func:`randn_` of a [B,C,H,W] tensor at ``noise_site``, ``x_t = q_sample(x0, t,
    eps)``; ``x0`` = the pool images."""
    if _hip(pool):
        ctr, off = idx_step if idx_step is not None else (None, 0)
        return _ops().gauss_batch(pool, rng, site, noise_site, total_steps, x_t, x0, t, idx, bool(draw_idx), ctr,
                                  int(off))
    salt = ref.site_salt(rng, site)
    B = x_t.shape[0]
    b = torch.arange(B, dtype=torch.int64)
    idx = stepped_idx(idx, idx_step, B)
    if draw_idx:
        idx.copy_(ref.mix32(ref._mul32((2 * b) & ref.MASK32, ref.GOLDEN) ^ salt) % pool.shape[0])
    t.copy_(ref.mix32(ref._mul32((2 * b + 1) & ref.MASK32, ref.GOLDEN) ^ salt) % total_steps)
    eps = torch.empty_like(x_t)
    randn_(eps, rng, noise_site)
    torch.index_select(pool, 0, idx, out=x0)
    x_t.copy_(ref.q_sample(x0, t, eps, total_steps))


def cold_batch(pool, rng, site: int, x_t, x_tm1, t, idx_ws, max_t: int, draw_idx: bool = True, idx_step=None):
    """Cold pixelation batch on device: t ~ U{1..max_t} (and pool indices unless
    ``draw_idx`` is False, in which case ``idx_ws`` holds them; ``idx_step``: see
    :func:`stepped_idx`), x_t / x_{t-1}."""
    if _hip(pool):
        ctr, off = idx_step if idx_step is not None else (None, 0)
        return _ops().cold_batch(pool, rng, site, x_t, x_tm1, t, idx_ws, max_t, bool(draw_idx), ctr, int(off))
    salt = ref.site_salt(rng, site)
    B = x_t.shape[0]
    b = torch.arange(B, dtype=torch.int64)
    idx_ws = stepped_idx(idx_ws, idx_step, B)
    if draw_idx:
        idx_ws.copy_(ref.mix32(ref._mul32((2 * b) & ref.MASK32, ref.GOLDEN) ^ salt) % pool.shape[0])
    t.copy_(1 + ref.mix32(ref._mul32((2 * b + 1) & ref.MASK32, ref.GOLDEN) ^ salt) % max_t)
    a, c = pixelate_pair(pool, idx_ws, t, B)
    x_t.copy_(a)
    x_tm1.copy_(c)
