"""The fused ViT program: explicit forward and hand-written backward.

Instead of a tracing compiler, the denoiser is a fixed sequence of fused HIP
ops (see :mod:`ddim_cold_amd.ops`), ~7 launches per transformer block forward
and ~11 backward, whose activations are saved explicitly.  The same program
object serves:

* :func:`fused_vit_forward` — an autograd Function so ``model(x, t)`` +
  ``loss.backward()`` work for library users (API parity with
  ``ViT.py:208-218``),
* :class:`ddim_cold_amd.train.engine.TrainEngine` — graph-captured training
  steps with flat parameter/gradient arenas, wgrad GEMMs on a side stream and
  bucketed RCCL all-reduce between backward segments,
* the samplers (forward-only, eval mode, hipGraph-captured loops).

Dropout sites: each dropout / drop-path application has a fixed integer site
id; masks are a pure function of (seed, step, site, element index) so the
backward regenerates exactly the forward's masks (no mask tensors stored).
Reference dropout placement: ``ViT.py:82,101,103,127,137,175``.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import Callable, Dict, Iterator, List, Optional

import torch

from .. import ops

SITE_EMBED = 1
FUSE_LN = os.environ.get("DDIM_COLD_FUSE_LN", "0") == "1"  # residual GEMM + LayerNorm in one kernel
# K split of the QKV input-gradient GEMM (reduction dim 3D): the partial products
# go to separate buffers that the LayerNorm backward sums on load
QKV_DGRAD_SPLITS = int(os.environ.get("DDIM_COLD_QKV_DGRAD_SPLITS", "2"))


def block_sites(i: int):
    s = 16 + 8 * i
    # attn-prob dropout, proj dropout, drop-path(attn), fc1(post-GELU) dropout, fc2 dropout, drop-path(mlp)
    return s, s + 1, s + 2, s + 3, s + 4, s + 5


@dataclass
class BlockTensors:
    n1w: torch.Tensor
    n1b: torch.Tensor
    qkv_w: torch.Tensor
    qkv_b: torch.Tensor
    proj_w: torch.Tensor
    proj_b: torch.Tensor
    n2w: torch.Tensor
    n2b: torch.Tensor
    fc1_w: torch.Tensor
    fc1_b: torch.Tensor
    fc2_w: torch.Tensor
    fc2_b: torch.Tensor


@dataclass
class ModelTensors:
    """Parameters (matrix weights in bf16) or gradients (all fp32) of one model."""
    cls: torch.Tensor
    pos: torch.Tensor
    pe_w: torch.Tensor
    pe_b: torch.Tensor
    temb: Optional[torch.Tensor]
    blocks: List[BlockTensors]
    nw: torch.Tensor
    nb: torch.Tensor
    head_w: torch.Tensor
    head_b: torch.Tensor


MATRIX_SUFFIXES = ("attn.qkv.weight", "attn.proj.weight", "mlp.fc1.weight", "mlp.fc2.weight")


def is_matrix_param(name: str) -> bool:
    return name == "patch_embed.proj.weight" or name == "head.weight" or name.endswith(MATRIX_SUFFIXES)


def collect(named: Dict[str, torch.Tensor], depth: int, D: int) -> ModelTensors:
    """Map reference parameter names to the program's tensor structure."""
    def g(n):
        return named.get(n)
    blocks = []
    for i in range(depth):
        p = f"blocks.{i}."
        blocks.append(BlockTensors(
            g(p + "norm1.weight"), g(p + "norm1.bias"), g(p + "attn.qkv.weight"), g(p + "attn.qkv.bias"),
            g(p + "attn.proj.weight"), g(p + "attn.proj.bias"), g(p + "norm2.weight"), g(p + "norm2.bias"),
            g(p + "mlp.fc1.weight"), g(p + "mlp.fc1.bias"), g(p + "mlp.fc2.weight"), g(p + "mlp.fc2.bias")))
    pe_w = g("patch_embed.proj.weight")
    return ModelTensors(
        cls=g("cls_token").reshape(D), pos=g("pos_embed").reshape(-1, D),
        pe_w=pe_w.reshape(pe_w.shape[0], -1) if pe_w is not None else None,
        pe_b=g("patch_embed.proj.bias"), temb=g("time_embed.weight"), blocks=blocks,
        nw=g("norm.weight"), nb=g("norm.bias"), head_w=g("head.weight"), head_b=g("head.bias"))


@dataclass
class ProgramConfig:
    img_h: int
    img_w: int
    patch: int
    chans: int
    dim: int
    depth: int
    heads: int
    hidden: int
    total_steps: int
    scale: float
    drop: float
    attn_drop: float
    dpr: List[float]
    eps: float = 1e-5
    learn_temb: bool = True

    @property
    def tokens(self) -> int:
        return (self.img_h // self.patch) * (self.img_w // self.patch) + 1

    @property
    def feat(self) -> int:
        return self.chans * self.patch * self.patch


@dataclass
class Saved:
    t: torch.Tensor
    patches: torch.Tensor
    blocks: list = field(default_factory=list)
    xL: Optional[torch.Tensor] = None
    lf: Optional[torch.Tensor] = None
    mf: Optional[torch.Tensor] = None
    rf: Optional[torch.Tensor] = None


def immediate_wgrad(dy, x, dw, db):
    ops.linear_wgrad(dy, x, dw, db)


class ViTProgram:
    def __init__(self, cfg: ProgramConfig):
        self.cfg = cfg

    @staticmethod
    def config_of(model) -> ProgramConfig:
        blk = model.blocks[0]
        return ProgramConfig(
            img_h=model.img_size[0], img_w=model.img_size[1], patch=model.patch_size, chans=model.in_chans,
            dim=model.embed_dim, depth=len(model.blocks), heads=model.num_heads,
            hidden=blk.mlp.fc1.out_features, total_steps=model.total_steps, scale=float(blk.attn.scale),
            drop=model.drop_rate, attn_drop=model.attn_drop_rate, dpr=model.drop_path_probs(),
            eps=float(blk.norm1.eps), learn_temb=model.time_embed.weight.requires_grad)

    @classmethod
    def from_model(cls, model) -> "ViTProgram":
        return cls(cls.config_of(model))

    def matches(self, model) -> bool:
        return self.config_of(model) == self.cfg

    # ------------------------------------------------------------------ forward
    def forward(self, P: ModelTensors, img: torch.Tensor, t: torch.Tensor, rng: torch.Tensor, training: bool,
                save: bool = True, head_step=None):
        """``head_step = (mode, x0_out, coef)`` fuses the sampler update into the head
        GEMM (``ops.head_step_``): ``img`` (the current x_t) is updated in place and
        returned; mode 1 = DDIM step, mode 2 = clamp (cold sampler)."""
        c = self.cfg
        B = img.shape[0]
        N, D, M = c.tokens, c.dim, B * c.tokens
        pd = c.drop if training else 0.0
        ad = c.attn_drop if training else 0.0
        dpr = c.dpr if training else [0.0] * c.depth
        x, patches = ops.patch_embed_fwd(img, t, P.pe_w, P.pe_b, P.cls, P.pos, P.temb, rng, SITE_EMBED, pd,
                                         c.patch)
        x = x.view(M, D)
        S = Saved(t=t, patches=patches) if save else None
        # Each residual GEMM carries the LayerNorm that follows it (proj -> norm2,
        # fc2 -> next block's norm1 / the final norm): ops.linear_residual_ln_fwd.
        # Off by default: the row-panel kernel concentrates the epilogue traffic on
        # M/32 workgroups and measured slower than GEMM + LayerNorm (15.5 vs 9.3 us
        # at M=2080; profiles/README.md).  DDIM_COLD_FUSE_LN=1 enables it.
        fuse = FUSE_LN and ops.residual_ln_fusable(D, D) and ops.residual_ln_fusable(D, c.hidden)
        l1, m1, r1 = ops.layernorm_fwd(x, P.blocks[0].n1w, P.blocks[0].n1b, c.eps)
        L = len(P.blocks)
        for i, bp in enumerate(P.blocks):
            sa, sp, sd1, sf1, sf2, sd2 = block_sites(i)
            x0 = x
            qkv = ops.qkv_fwd(l1, bp.qkv_w, bp.qkv_b, B, N, c.heads)
            o, lse = ops.attn_fwd(qkv, c.scale, rng, sa, ad)
            o = o.view(M, D)
            if fuse:
                x1, l2, m2, r2 = ops.linear_residual_ln_fwd(o, bp.proj_w, bp.proj_b, x0, bp.n2w, bp.n2b, c.eps, N,
                                                            rng, sp, pd, sd1, dpr[i])
            else:
                x1 = ops.linear_residual_fwd(o, bp.proj_w, bp.proj_b, x0, N, rng, sp, pd, sd1, dpr[i])
                l2, m2, r2 = ops.layernorm_fwd(x1, bp.n2w, bp.n2b, c.eps)
            u, h = ops.linear_gelu_fwd(l2, bp.fc1_w, bp.fc1_b, rng, sf1, pd)
            nw, nb = (P.blocks[i + 1].n1w, P.blocks[i + 1].n1b) if i + 1 < L else (P.nw, P.nb)
            if fuse:
                x, ln_n, m_n, r_n = ops.linear_residual_ln_fwd(h, bp.fc2_w, bp.fc2_b, x1, nw, nb, c.eps, N, rng, sf2,
                                                               pd, sd2, dpr[i])
            else:
                x = ops.linear_residual_fwd(h, bp.fc2_w, bp.fc2_b, x1, N, rng, sf2, pd, sd2, dpr[i])
                ln_n, m_n, r_n = ops.layernorm_fwd(x, nw, nb, c.eps)
            if save:
                S.blocks.append((x0, l1, m1, r1, qkv, o, lse, x1, l2, m2, r2, u, h))
            l1, m1, r1 = ln_n, m_n, r_n
        lf, mf, rf = l1, m1, r1
        if head_step is not None:
            mode, x0_out, coef = head_step
            ops.head_step_(lf, P.head_w, P.head_b, img, x0_out, coef, c.patch, mode)
            return img, S
        out = ops.head_fwd(lf, P.head_w, P.head_b, B, c.chans, c.img_h, c.img_w, c.patch)
        if save:
            S.xL, S.lf, S.mf, S.rf = x, lf, mf, rf
        return out, S

    # ------------------------------------------------------------------ backward
    def backward_iter(self, P: ModelTensors, G: ModelTensors, S: Saved, dtok: torch.Tensor, rng: torch.Tensor,
                      training: bool = True, wgrad: Optional[Callable] = None,
                      ln_ws: Optional[torch.Tensor] = None, wgrad_stream=None) -> Iterator[int]:
        """Hand-written backward; yields the block index after each block's grads
        are issued (L-1 first, then ..., 0) and -1 after the embedding grads.

        ``G`` tensors are fp32 accumulators (``+=``).  By default the weight
        gradients of each block (qkv, proj, fc1, fc2; plus the head with the
        last block) are batched and issued as ONE grouped GEMM launch at the end
        of the block (``ops.WgradBatch``); a ``wgrad`` callable instead issues
        each one immediately (e.g. on a side stream).  ``ln_ws`` ([2L+1, R, 2D],
        zero) collects LayerNorm dgamma/dbeta replicas in backward order (final
        norm, then norm2/norm1 of blocks L-1..0); the caller finalises them
        with ``ops.replica_reduce_``.
        """
        def ws(k):
            return None if ln_ws is None else ln_ws[k]
        batch = None
        if wgrad is None:
            batch = wgrad = ops.WgradBatch(wgrad_stream)

        def flush():
            if batch is not None:
                batch.flush()
        c = self.cfg
        N, D = c.tokens, c.dim
        pd = c.drop if training else 0.0
        ad = c.attn_drop if training else 0.0
        dpr = c.dpr if training else [0.0] * c.depth
        L = c.depth
        dlf = ops.linear_dgrad(dtok, P.head_w, True)
        wgrad(dtok, S.lf, G.head_w, G.head_b)
        _, _, _, _, sf2, sd2 = block_sites(L - 1)
        g, gy = ops.layernorm_bwd(dlf, S.xL, S.mf, S.rf, P.nw, None, G.nw, G.nb, N, rng, sf2, pd, sd2,
                                  dpr[L - 1], True, ws(0))
        keep = []
        for i in range(L - 1, -1, -1):
            x0, l1, m1, r1, qkv, o, lse, x1, l2, m2, r2, u, h = S.blocks[i]
            bp, bg = P.blocks[i], G.blocks[i]
            sa, sp, sd1, sf1, _, _ = block_sites(i)
            wgrad(gy, h, bg.fc2_w, bg.fc2_b)
            du = ops.linear_dgrad_gelu(gy, bp.fc2_w, u, rng, sf1, pd)
            wgrad(du, l2, bg.fc1_w, bg.fc1_b)
            dl2 = ops.linear_dgrad(du, bp.fc1_w, True)
            k2 = 1 + 2 * (L - 1 - i)
            g1, gy1 = ops.layernorm_bwd(dl2, x1, m2, r2, bp.n2w, g, bg.n2w, bg.n2b, N, rng, sp, pd, sd1, dpr[i],
                                        True, ws(k2))
            wgrad(gy1, o, bg.proj_w, bg.proj_b)
            do = ops.linear_dgrad(gy1, bp.proj_w, False)
            dqkv = ops.attn_bwd(do, qkv, o, lse, c.scale, rng, sa, ad)
            wgrad(dqkv, l1, bg.qkv_w, bg.qkv_b)
            dl1 = ops.linear_dgrad(dqkv, bp.qkv_w, True, QKV_DGRAD_SPLITS if 3 * D >= 768 else 1)
            if i > 0:
                _, _, _, _, psf2, psd2 = block_sites(i - 1)
                g, gy = ops.layernorm_bwd(dl1, x0, m1, r1, bp.n1w, g1, bg.n1w, bg.n1b, N, rng, psf2, pd, psd2,
                                          dpr[i - 1], True, ws(k2 + 1))
            else:
                g, gy = ops.layernorm_bwd(dl1, x0, m1, r1, bp.n1w, g1, bg.n1w, bg.n1b, N, rng, 0, 0.0, 0, 0.0,
                                          False, ws(k2 + 1))
            keep.append((gy1, du, dqkv))
            flush()
            yield i
        B = S.t.shape[0]
        temb_g = G.temb if G.temb is not None else torch.zeros_like(P.temb)
        gpatch = ops.embed_bwd(g.view(B, N, D), S.t, rng, SITE_EMBED, pd, G.cls, G.pos, temb_g)
        wgrad(gpatch, S.patches, G.pe_w, G.pe_b)
        flush()
        keep.append(gpatch)
        if batch is not None:
            keep.append(batch.keep)
        self._keep = keep  # holds side-stream operands alive until the caller joins
        yield -1

    def backward(self, P, G, S, dtok, rng, training=True, wgrad=None):
        for _ in self.backward_iter(P, G, S, dtok, rng, training, wgrad):
            pass
        self._keep = None


# ---------------------------------------------------------------------- autograd wrapper
def _bf16_cached(model, name: str, p: torch.Tensor) -> torch.Tensor:
    cache = model.__dict__.setdefault("_bf16_cache", {})
    key = (p.data_ptr(), p._version, p.device)
    hit = cache.get(name)
    if hit is not None and hit[0] == key:
        return hit[1]
    w = p.detach().to(torch.bfloat16).contiguous()
    cache[name] = (key, w)
    return w


def model_tensors(model, named: Optional[Dict[str, torch.Tensor]] = None) -> ModelTensors:
    """Program parameter view of ``model``: fp32 params, bf16 matrix weights.

    If a training engine owns the model (flat arenas + bf16 shadow maintained
    by the fused optimizer) its views are used directly.
    """
    eng = getattr(model, "_engine", None)
    if eng is not None:
        return eng.param_tensors
    named = named if named is not None else dict(model.named_parameters())
    conv = {}
    for n, p in named.items():
        conv[n] = _bf16_cached(model, n, p) if is_matrix_param(n) else p.detach()
    return collect(conv, len(model.blocks), model.embed_dim)


def rng_state(model, device) -> torch.Tensor:
    eng = getattr(model, "_engine", None)
    if eng is not None:
        return eng.rng
    st = model.__dict__.get("_rng_state")
    if st is None or st.device != torch.device(device):
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        st = torch.tensor([seed, 0], dtype=torch.int64, device=device)
        model.__dict__["_rng_state"] = st
    return st


class _FusedViT(torch.autograd.Function):
    @staticmethod
    def forward(ctx, model, img, t, *params):
        prog = model.program()
        names = [n for n, _ in model.named_parameters()]
        P = model_tensors(model, dict(zip(names, params)))
        rng = rng_state(model, img.device)
        if model.training:
            rng[1] += 1  # fresh dropout masks per call (device-side increment)
        rng_snap = rng.clone()
        out, S = prog.forward(P, img.contiguous(), t.contiguous(), rng_snap, model.training,
                              save=torch.is_grad_enabled() or any(ctx.needs_input_grad))
        ctx.model, ctx.prog, ctx.S, ctx.P, ctx.rng = model, prog, S, P, rng_snap
        ctx.names, ctx.training = names, model.training
        ctx.shapes = [p.shape for p in params]
        return out

    @staticmethod
    def backward(ctx, dimg):
        prog, S, P = ctx.prog, ctx.S, ctx.P
        c = prog.cfg
        grads = {n: torch.zeros(s, dtype=torch.float32, device=dimg.device) for n, s in zip(ctx.names, ctx.shapes)}
        G = collect(grads, c.depth, c.dim)
        dtok = ops.img_to_tokgrad(dimg.float().contiguous(), c.tokens, c.patch)
        prog.backward(P, G, S, dtok, ctx.rng, ctx.training)
        ctx.S = None
        out = [grads[n] if ctx.needs_input_grad[3 + i] else None for i, n in enumerate(ctx.names)]
        return (None, None, None, *out)


def fused_vit_forward(model, x: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
    params = [p for _, p in model.named_parameters()]
    if x.dtype != torch.float32:
        x = x.float()
    return _FusedViT.apply(model, x, t.long(), *params)
