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
# K split of the QKV input-gradient GEMM (reduction dim 3D; the partial products go to
# separate buffers that the LayerNorm backward sums on load).  Unsplit measured best at
# every model size this round (tools/ab_module_constant.py, two interleaved reps each:
# ViT-tiny 0.7349 / 0.7348 ms/step unsplit vs 0.7386 / 0.7358 with 2 and 0.7475 / 0.7357
# with 3; vit_small_200 6.523 / 6.541 vs 6.578 / 6.610 with 2)
QKV_DGRAD_SPLITS = 1
# the input-gradient GEMMs feeding a LayerNorm backward (head, fc1, QKV) write
# bf16 (the K-split partials too) instead of fp32: half the bytes on both sides
# of the dgrad -> LayerNorm-backward hand-off; the LayerNorm backward sums and
# computes in fp32 (the reference's fp16 autocast hands it fp16 gradients)
DGRAD_BF16 = True
# LayerNorm backward of a folded LayerNorm reads the bf16 copy of its input -- the
# operand the folded GEMM normalised in the forward -- instead of the fp32 residual
# stream: 2 of its 18 bytes per element, and the fp32 block inputs are not saved
LN_BWD_XB = True
# GEMMs per LayerNorm-fold launch (csrc/kernels.h FOLD_MAX)
FOLD_MAX = 32
# LayerNorm fold (csrc/gemm.hip): every LayerNorm is folded into the GEMM that
# consumes it (QKV, fc1, head) -- no LayerNorm launch in the forward.  The
# producing GEMM's epilogue accumulates the row statistics; the LayerNorm
# backward re-emits the normalised rows for the weight gradients.
FOLD_LN = True  # False: separate LayerNorm launches (tests compare both)
# the short attention forward stores its dropout keep flags (one 32-bit word per
# lane, 0.6 MB per block for ViT-tiny at B=32) and the backward reads them instead
# of re-hashing 2 pairs per 4 probabilities (the mask hash was ~1.9 us of the
# backward's ~11 us, tools/ub_drop.py).  Same masks either way.
STORE_ATTN_KEEP = True
# training with the fused batch draw: loss target as patch rows, vector loss epilogue
# (EPI_HEADL; head GEMM 11.3 -> see profiles/README.md round 3)
TARGET_ROWS = True
# dtype of the bf16 activation copies / folded weights the program allocates
# (tests on CPU switch it to fp32 to isolate the program logic from rounding)
ACT_DTYPE = torch.bfloat16


def fold_width_ok(D: int) -> bool:
    """Widths the LayerNorm fold supports (csrc/gemm.hip: 32-column statistics slots, <= 16)."""
    return D % 32 == 0 and D // 32 <= 16


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
    # LayerNorm fold (LnFold.attach): gamma-scaled bf16 weight, its row sums, folded bias
    qkv_wf: Optional[torch.Tensor] = None
    qkv_c: Optional[torch.Tensor] = None
    qkv_bf: Optional[torch.Tensor] = None
    fc1_wf: Optional[torch.Tensor] = None
    fc1_c: Optional[torch.Tensor] = None
    fc1_bf: Optional[torch.Tensor] = None
    # transposed bf16 shadows ([in][out]) for the input-gradient GEMMs (train engine,
    # long sequences: TransposedShadows): dX = dY W on the k-contiguous operand path
    qkv_wt: Optional[torch.Tensor] = None
    proj_wt: Optional[torch.Tensor] = None
    fc1_wt: Optional[torch.Tensor] = None
    fc2_wt: Optional[torch.Tensor] = None


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
    head_wf: Optional[torch.Tensor] = None
    head_c: Optional[torch.Tensor] = None
    head_bf: Optional[torch.Tensor] = None

    @property
    def folded(self) -> bool:
        return self.head_wf is not None


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


class LnFold:
    """Folded weights of every GEMM that consumes a LayerNorm (QKV <- norm1,
    fc1 <- norm2, head <- norm), in three flat arenas; :meth:`refresh` recomputes
    them from the fp32 masters in one ``ln_fold_`` launch per 16 GEMMs (after
    every optimizer step in the train engine; once per weight version for
    inference)."""

    @staticmethod
    def jobs(depth: int):
        """(key, weight, gamma, beta, bias) parameter names of every folded GEMM."""
        jobs = []
        for i in range(depth):
            p = f"blocks.{i}."
            jobs.append((("qkv", i), p + "attn.qkv.weight", p + "norm1.weight", p + "norm1.bias", p + "attn.qkv.bias"))
            jobs.append((("fc1", i), p + "mlp.fc1.weight", p + "norm2.weight", p + "norm2.bias", p + "mlp.fc1.bias"))
        jobs.append((("head",), "head.weight", "norm.weight", "norm.bias", "head.bias"))
        return jobs

    @staticmethod
    def names(depth: int):
        return [n for j in LnFold.jobs(depth) for n in j[1:]]

    def __init__(self, named32: Dict[str, torch.Tensor], depth: int,
                 weights: Optional[Dict[str, torch.Tensor]] = None):
        """``weights``: optional replacement tensors for the matrix weights (the
        engine passes its bf16 shadow copies: the fold then reads half the bytes)."""
        jobs = self.jobs(depth)
        self.keys = [j[0] for j in jobs]
        self.src = [tuple((weights[n] if (weights is not None and k == 0) else named32[n])
                          for k, n in enumerate(j[1:])) for j in jobs]
        w0 = self.src[0][0]
        dev, K = w0.device, w0.shape[1]
        rows = [w.shape[0] for w, _, _, _ in self.src]
        # 16-B aligned sub-ranges (vector loads/stores in the GEMMs)
        offs, o = [], 0
        for r in rows:
            offs.append(o)
            o += (r + 7) // 8 * 8
        self.wf_arena = torch.zeros(o * K, dtype=ACT_DTYPE, device=dev)
        self.c_arena = torch.zeros(o, dtype=torch.float32, device=dev)
        self.bf_arena = torch.zeros(o, dtype=torch.float32, device=dev)
        self.out = {}
        for key, r, off in zip(self.keys, rows, offs):
            self.out[key] = (self.wf_arena[off * K:(off + r) * K].view(r, K), self.c_arena[off:off + r],
                             self.bf_arena[off:off + r])

    def tensors(self):
        return [t for w, g, b, bias in self.src for t in (w, g, b, bias)]

    def refresh(self, tail=None):
        """Recompute the folded weights; ``tail`` (see :func:`ops.ln_fold_`) rides
        along in the last launch."""
        for a in range(0, len(self.keys), FOLD_MAX):
            ks = self.keys[a:a + FOLD_MAX]
            src = self.src[a:a + FOLD_MAX]
            last = a + FOLD_MAX >= len(self.keys)
            ops.ln_fold_([w.reshape(w.shape[0], -1) for w, _, _, _ in src], [g for _, g, _, _ in src],
                         [b for _, _, b, _ in src], [bias for _, _, _, bias in src],
                         [self.out[k][0] for k in ks], [self.out[k][1] for k in ks], [self.out[k][2] for k in ks],
                         tail=tail if last else None)

    def attach(self, P: "ModelTensors") -> "ModelTensors":
        for i, bp in enumerate(P.blocks):
            bp.qkv_wf, bp.qkv_c, bp.qkv_bf = self.out[("qkv", i)]
            bp.fc1_wf, bp.fc1_c, bp.fc1_bf = self.out[("fc1", i)]
        P.head_wf, P.head_c, P.head_bf = self.out[("head",)]
        return P


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
    keeps: list = field(default_factory=list)  # per block: stored attention keep flags or None
    xL: Optional[torch.Tensor] = None
    lf: Optional[torch.Tensor] = None
    mf: Optional[torch.Tensor] = None
    rf: Optional[torch.Tensor] = None


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
                save: bool = True, head_step=None, loss=None, cold=None):
        """``head_step = (mode, x0_out, coef)`` fuses the sampler update into the head
        GEMM (``ops.head_step_``): ``img`` (the current x_t) is updated in place and
        returned; mode 1 = DDIM step, mode 2 = clamp (cold sampler).  ``loss =
        (target, beta)`` (LayerNorm-folded program only, see :meth:`supports_fused_loss`)
        returns ``(loss_parts, dtok)`` from :func:`ops.head_loss` instead of the image.
        ``cold`` (LayerNorm-folded program only): the cold batch draw fused into the
        patch embedding (:func:`ops.patch_embed_cold_fwd`); ``img``/``t`` are its outputs."""
        if P.folded and fold_width_ok(self.cfg.dim):
            return self._forward_folded(P, img, t, rng, training, save, head_step, loss, cold)
        if loss is not None or cold is not None:
            raise ValueError("the fused head loss / cold batch need the LayerNorm-folded program")
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
        l1, m1, r1 = ops.layernorm_fwd(x, P.blocks[0].n1w, P.blocks[0].n1b, c.eps)
        L = len(P.blocks)
        for i, bp in enumerate(P.blocks):
            sa, sp, sd1, sf1, sf2, sd2 = block_sites(i)
            x0 = x
            qkv = ops.qkv_fwd(l1, bp.qkv_w, bp.qkv_b, B, N, c.heads)
            o, lse = ops.attn_fwd(qkv, c.scale, rng, sa, ad)
            o = o.view(M, D)
            x1 = ops.linear_residual_fwd(o, bp.proj_w, bp.proj_b, x0, N, rng, sp, pd, sd1, dpr[i])
            l2, m2, r2 = ops.layernorm_fwd(x1, bp.n2w, bp.n2b, c.eps)
            u, h = ops.linear_gelu_fwd(l2, bp.fc1_w, bp.fc1_b, rng, sf1, pd)
            nw, nb = (P.blocks[i + 1].n1w, P.blocks[i + 1].n1b) if i + 1 < L else (P.nw, P.nb)
            x = ops.linear_residual_fwd(h, bp.fc2_w, bp.fc2_b, x1, N, rng, sf2, pd, sd2, dpr[i])
            ln_n, m_n, r_n = ops.layernorm_fwd(x, nw, nb, c.eps)
            if save:
                S.blocks.append((x0, l1, m1, r1, qkv, o, lse, x1, l2, m2, r2, u, h))
            l1, m1, r1 = ln_n, m_n, r_n
        lf, mf, rf = l1, m1, r1
        if head_step is not None:
            mode, x0_out, coef = head_step[:3]  # (patch-row hand-off: folded forward only)
            ops.head_step_(lf, P.head_w, P.head_b, img, x0_out, coef, c.patch, mode)
            return img, S
        out = ops.head_fwd(lf, P.head_w, P.head_b, B, c.chans, c.img_h, c.img_w, c.patch)
        if save:
            S.xL, S.lf, S.mf, S.rf = x, lf, mf, rf
        return out, S

    def _forward_folded(self, P: ModelTensors, img, t, rng, training: bool, save: bool, head_step, loss=None,
                        cold=None):
        """Forward with every LayerNorm folded into its consumer GEMM: 5 launches
        per block (QKV, attention, proj+residual, fc1+GELU, fc2+residual).  The
        residual GEMMs (and the patch embedding) emit each new residual row's
        {sum, sum^2} and bf16 copy; QKV / fc1 / head read that copy with
        gamma-scaled weights and apply mean / rstd in their epilogue.  Saved
        tensors match the unfolded forward except the LayerNorm outputs (None:
        the backward re-emits them)."""
        c = self.cfg
        B = img.shape[0]
        N, D, M, L = c.tokens, c.dim, B * c.tokens, c.depth
        pd = c.drop if training else 0.0
        ad = c.attn_drop if training else 0.0
        dpr = c.dpr if training else [0.0] * c.depth
        dev = img.device
        # row statistics of every LayerNorm input ({sum, sum^2} per 32-column slot),
        # each slot written once by the producing epilogue
        st = torch.empty(2 * L + 1, M, D // 32, 2, dtype=torch.float32, device=dev)
        xb = torch.empty(M, D, dtype=ACT_DTYPE, device=dev)
        # sampler steps: head_step = (mode, x0_out, coef, patches_in, patches_out[,
        # pe_w_rows]); the previous step's head left this step's bf16 patch rows in
        # patches_in.  With pe_w_rows the sampler state lives in patch rows
        # (ops.image_to_rows; ``img`` is a [B, C, H, W]-shaped view of that buffer):
        # the embedding reads the rows through the column-permuted weight and the
        # head updates them with contiguous vector accesses (ops.head_step_rows_)
        patches_in = head_step[3] if head_step is not None and len(head_step) > 3 else None
        rows_w = head_step[5] if head_step is not None and len(head_step) > 5 else None
        if rows_w is not None and patches_in is None:
            raise ValueError("the patch-row sampler state needs patches_in")
        # the fused batch draw writes the loss target as patch rows for the vector
        # loss epilogue (ops.head_loss target_rows; the target buffer is only read there)
        tgt_rows = cold is not None and loss is not None and TARGET_ROWS
        if cold is not None:
            x, patches = ops.patch_embed_cold_fwd(cold, img, t, P.pe_w, P.pe_b, P.cls, P.pos, P.temb, rng,
                                                  SITE_EMBED, pd, c.patch, ln_st=st[0], xb_out=xb,
                                                  target_rows=tgt_rows)
        else:
            x, patches = ops.patch_embed_fwd(img, t, P.pe_w if rows_w is None else rows_w, P.pe_b, P.cls, P.pos,
                                             P.temb, rng, SITE_EMBED, pd, c.patch, ln_st=st[0], xb_out=xb,
                                             patches_in=patches_in)
        x = x.view(M, D)
        S = Saved(t=t, patches=patches) if save else None

        def stats():
            return (torch.empty(M, dtype=torch.float32, device=dev),
                    torch.empty(M, dtype=torch.float32, device=dev)) if save else (None, None)
        for i, bp in enumerate(P.blocks):
            sa, sp, sd1, sf1, sf2, sd2 = block_sites(i)
            x0, x0b = x, xb
            m1, r1 = stats()
            fold = (st[2 * i], bp.qkv_c, c.eps, m1, r1)
            qkv = ops.qkv_fwd(xb, bp.qkv_wf, bp.qkv_bf, B, N, c.heads, fold=fold)
            keep = ops.attn_keep_buffer(qkv, ad) if save and STORE_ATTN_KEEP else None
            o, lse = ops.attn_fwd(qkv, c.scale, rng, sa, ad, keep_out=keep)
            if save:
                S.keeps.append(keep)
            o = o.view(M, D)
            x1b = torch.empty(M, D, dtype=ACT_DTYPE, device=dev)
            x1 = ops.linear_residual_fwd(o, bp.proj_w, bp.proj_b, x0, N, rng, sp, pd, sd1, dpr[i],
                                         st_out=st[2 * i + 1], xb_out=x1b)
            m2, r2 = stats()
            xb = torch.empty(M, D, dtype=ACT_DTYPE, device=dev)
            u, h = ops.linear_gelu_fwd(x1b, bp.fc1_wf, bp.fc1_bf, rng, sf1, pd,
                                       fold=(st[2 * i + 1], bp.fc1_c, c.eps, m2, r2))
            x = ops.linear_residual_fwd(h, bp.fc2_w, bp.fc2_b, x1, N, rng, sf2, pd, sd2, dpr[i],
                                        st_out=st[2 * i + 2], xb_out=xb)
            if save:
                # the LayerNorm backwards read the bf16 copies the folded GEMMs normalised
                xs0, xs1 = (x0b, x1b) if LN_BWD_XB else (x0, x1)
                S.blocks.append((xs0, None, m1, r1, qkv, o, lse, xs1, None, m2, r2, u, h))
        if head_step is not None:
            mode, x0_out, coef = head_step[:3]
            patches_out = head_step[4] if len(head_step) > 4 else None
            if rows_w is not None:
                F = P.head_wf.shape[0]
                ops.head_step_rows_(xb, P.head_wf, P.head_bf, img.view(-1, F),
                                    None if x0_out is None else x0_out.view(-1, F), coef, B, mode,
                                    patches_out=patches_out, fold=(st[2 * L], P.head_c, c.eps))
                return img, S
            ops.head_step_(xb, P.head_wf, P.head_bf, img, x0_out, coef, c.patch, mode, patches_out=patches_out,
                           fold=(st[2 * L], P.head_c, c.eps))
            return img, S
        mf, rf = stats()
        if loss is not None:  # training: the loss and its token-layout gradient from the head GEMM
            target, beta = loss
            out = ops.head_loss(xb, P.head_wf, P.head_bf, target, c.patch, beta,
                                fold=(st[2 * L], P.head_c, c.eps, mf, rf), target_rows=tgt_rows)
        else:
            out = ops.head_fwd(xb, P.head_wf, P.head_bf, B, c.chans, c.img_h, c.img_w, c.patch,
                               fold=(st[2 * L], P.head_c, c.eps, mf, rf))
        if save:
            S.xL, S.lf, S.mf, S.rf = xb if LN_BWD_XB else x, None, mf, rf
        return out, S

    def supports_fused_loss(self, P: ModelTensors) -> bool:
        return P.folded and fold_width_ok(self.cfg.dim)

    # ------------------------------------------------------------------ backward
    def backward_iter(self, P: ModelTensors, G: ModelTensors, S: Saved, dtok: torch.Tensor, rng: torch.Tensor,
                      training: bool = True, wgrad: Optional[Callable] = None,
                      ln_ws: Optional[torch.Tensor] = None, embed_with_block0: bool = False, ln_final=None,
                      wgrad_flush=None, wgrad_store: bool = False, wgrad_sq=None,
                      embed_fused=None) -> Iterator[int]:
        """Hand-written backward; yields the block index after each block's input
        gradients are issued (L-1 first, then ..., 0) and -1 after the embedding grads.

        ``G`` tensors are fp32 accumulators (``+=``).  Weight gradients are deferred:
        by default EVERY ``dW += dy^T x`` of the backward (4 per block, head, patch
        embedding) is queued and issued as ONE launch after the embedding backward
        (:func:`ops.linear_wgrad_multi`; nothing reads a block's gradients before the
        optimizer), so a block yield only marks the order.  ``wgrad_flush`` (a set of
        block indices; data parallel): one such launch per gradient bucket -- after
        each listed block and after the embedding backward -- so the bucket's
        all-reduce can start while the rest of the backward runs.  A ``wgrad``
        callable instead receives each job as soon as its operands exist.
        ``ln_ws`` ([2L+1, R, 2D], zero) collects LayerNorm dgamma/dbeta replicas in
        backward order (final norm, then norm2/norm1 of blocks L-1..0); the caller
        finalises them with ``ops.replica_reduce_`` (or ``ln_final``, carried by the
        embedding-backward launch).  ``embed_with_block0``: the embedding backward
        runs before block 0's weight gradients are flushed (no separate embedding
        bucket).  ``wgrad_store``: the block / head weight-gradient targets have no
        other writer this step, so the deferred launches write instead of
        read-add-writing them (the embedding bucket's patch gradient still adds).
        ``wgrad_sq = (parts, arena, lazy)`` (one deferred launch, no ``wgrad_flush``):
        that launch also writes the grad-norm partials of the whole gradient arena
        (:func:`ops.linear_wgrad_multi`), so the optimizer needs no sqnorm pass.
        ``embed_fused = (owners, ln_offs)`` (with ``wgrad_sq``): no embedding-backward
        launch -- the last LayerNorm backward writes the patch-row gradient and the
        cls / pos / time-embedding gradients and the LayerNorm finalize (``ln_final``,
        ``ln_offs`` = its destinations' arena offsets) run as extra workgroups of the
        weight-gradient launch (``owners`` >= the distinct timesteps of a batch).
        Measured slower on MI355X and removed: weight gradients riding in the
        input-gradient launches, one grouped launch per block, a side-stream branch
        for them, the proj input gradient inside the attention backward, the
        LayerNorm backward in the epilogue or the prologue of its neighbouring GEMM
        (profiles/fused_ln_qkv_r5_ab.txt, profiles/ln_prologue_r5.md)."""
        def ws(k):
            return None if ln_ws is None else ln_ws[k]
        bucketed = wgrad is None and wgrad_flush is not None
        if wgrad_sq is not None and (bucketed or wgrad is not None):
            raise ValueError("wgrad_sq needs the single deferred weight-gradient launch")
        if embed_fused is not None and (wgrad_sq is None or G.temb is None or not embed_with_block0):
            raise ValueError("embed_fused needs wgrad_sq, a trainable time embedding and embed_with_block0")
        emb_spec = None
        jobs = []
        if wgrad is None:
            wgrad = lambda dy, x, dw, db: jobs.append((dy, x, dw, db))  # noqa: E731
        c = self.cfg
        N, D = c.tokens, c.dim
        pd = c.drop if training else 0.0
        ad = c.attn_drop if training else 0.0
        dpr = c.dpr if training else [0.0] * c.depth
        L = c.depth
        M = dtok.shape[0]
        # LayerNorm fold: the forward never materialised the LayerNorm outputs;
        # each LayerNorm backward re-emits its output (bf16) for the weight
        # gradient queued right after it
        fold = S.lf is None

        def ln_out(lo):
            return torch.empty(M, D, dtype=ACT_DTYPE, device=dtok.device) if fold else lo
        f32 = not DGRAD_BF16
        keep = []

        def dgrad(dy, w, wt, out_f32, splits=1):
            """dy @ w; with the transposed shadow wt (= w.T) on the k-contiguous operand
            path (csrc/transpose.hip: 31.7 -> 25.5 us for vit_small_200's QKV)"""
            if wt is not None and splits == 1:
                return ops.linear_fwd(dy, wt, None, out_f32)
            return ops.linear_dgrad(dy, w, out_f32, splits)

        def dgrad_ln(dy, w, splits, x, *ln_args, wt=None, **ln_kw):
            """dy @ w, then the LayerNorm backward (keep: the bf16 hand-off stays referenced)"""
            dl = dgrad(dy, w, wt, f32, splits)
            keep.append(dl)
            return ops.layernorm_bwd(dl, x, *ln_args, **ln_kw)

        lf = ln_out(S.lf)
        _, _, _, _, sf2, sd2 = block_sites(L - 1)
        g, gy = dgrad_ln(dtok, P.head_w, 1, S.xL, S.mf, S.rf, P.nw, None, G.nw, G.nb, N, rng, sf2, pd, sd2,
                         dpr[L - 1], True, ws(0), beta=P.nb if fold else None, y_out=lf if fold else None)
        wgrad(dtok, lf, G.head_w, G.head_b)
        for i in range(L - 1, -1, -1):
            x0, l1, m1, r1, qkv, o, lse, x1, l2, m2, r2, u, h = S.blocks[i]
            bp, bg = P.blocks[i], G.blocks[i]
            sa, sp, sd1, sf1, _, _ = block_sites(i)
            du = ops.linear_dgrad_gelu(gy, bp.fc2_w, u, rng, sf1, pd, wt=bp.fc2_wt)
            wgrad(gy, h, bg.fc2_w, bg.fc2_b)
            k2 = 1 + 2 * (L - 1 - i)
            l2 = ln_out(l2)
            g1, gy1 = dgrad_ln(du, bp.fc1_w, 1, x1, m2, r2, bp.n2w, g, bg.n2w, bg.n2b, N, rng, sp, pd, sd1,
                               dpr[i], True, ws(k2), beta=bp.n2b if fold else None, y_out=l2 if fold else None,
                               wt=bp.fc1_wt)
            do = dgrad(gy1, bp.proj_w, bp.proj_wt, False)
            wgrad(du, l2, bg.fc1_w, bg.fc1_b)
            wgrad(gy1, o, bg.proj_w, bg.proj_b)
            dqkv = ops.attn_bwd(do, qkv, o, lse, c.scale, rng, sa, ad,
                                keep=S.keeps[i] if len(S.keeps) == L else None)
            qs = QKV_DGRAD_SPLITS if 3 * D >= 768 else 1
            l1 = ln_out(l1)
            fk = dict(beta=bp.n1b, y_out=l1) if fold else {}
            if i > 0:
                _, _, _, _, psf2, psd2 = block_sites(i - 1)
                g, gy = dgrad_ln(dqkv, bp.qkv_w, qs, x0, m1, r1, bp.n1w, g1, bg.n1w, bg.n1b, N, rng, psf2, pd, psd2,
                                 dpr[i - 1], True, ws(k2 + 1), wt=bp.qkv_wt, **fk)
            else:
                if embed_fused is not None:  # the patch-row gradient from this LayerNorm backward
                    Bs = S.t.shape[0]
                    gpatch = torch.empty(Bs * (N - 1), D, dtype=ACT_DTYPE, device=dtok.device)
                    fk = dict(fk, gp_out=gpatch, site_emb=SITE_EMBED, p_emb=pd)
                g, gy = dgrad_ln(dqkv, bp.qkv_w, qs, x0, m1, r1, bp.n1w, g1, bg.n1w, bg.n1b, N, rng, 0, 0.0, 0, 0.0,
                                 False, ws(k2 + 1), wt=bp.qkv_wt, **fk)
            keep.append((gy1, du, dqkv, l1, l2, do))
            wgrad(dqkv, l1, bg.qkv_w, bg.qkv_b)
            if i == 0 and embed_with_block0 and embed_fused is not None:
                wgrad(gpatch, S.patches, G.pe_w, G.pe_b)
                owners, ln_offs = embed_fused
                ln = None
                if ln_final is not None:
                    lw, lp, lC, lR = ln_final[:4]
                    ln = (lw, lp, ln_offs, lC, lR, bool(ln_final[4]) if len(ln_final) > 4 else False)
                emb_spec = (g.view(S.t.shape[0], N, D), S.t, rng, SITE_EMBED, pd, G.cls, G.pos, G.temb,
                            min(int(owners), S.t.shape[0]), ln)
            elif i == 0 and embed_with_block0:
                gpatch = self._embed_backward(P, G, S, g, rng, pd, wgrad, ln_final)
            if bucketed and (i in wgrad_flush or (i == 0 and embed_with_block0)) and jobs:
                ops.linear_wgrad_multi(jobs, store=wgrad_store)  # this bucket's weight gradients: final now
                keep.append(jobs)
                jobs = []
            yield i
        if not embed_with_block0:
            gpatch = self._embed_backward(P, G, S, g, rng, pd, wgrad, ln_final)
        if jobs:
            tiles = sum(-(-dy.shape[1] // 64) * -(-x.shape[1] // 64) for dy, x, _, _ in jobs)
            if bucketed and tiles < 64:
                # the embedding bucket's patch-embedding gradient alone (18 tiles for
                # ViT-tiny): unsplit, 18 workgroups walk all 2,048 tokens (~17 us on the
                # step's critical path); the token-split kernel fills the chip
                for job in jobs:
                    ops.linear_wgrad(*job)
            else:
                ops.linear_wgrad_multi(jobs, store=wgrad_store and not bucketed, sq=wgrad_sq, embed=emb_spec)
            keep.append(jobs)
        keep.append((gpatch, lf))
        self._keep = keep  # operands of the queued launches stay referenced until the next step
        yield -1

    def _embed_backward(self, P, G, S, g, rng, pd, wgrad, ln_final=None):
        """cls / pos / time-embedding gradients and the patch-embedding weight gradient (queued)."""
        c = self.cfg
        B = S.t.shape[0]
        temb_g = G.temb if G.temb is not None else torch.zeros_like(P.temb)
        gpatch = ops.embed_bwd(g.view(B, c.tokens, c.dim), S.t, rng, SITE_EMBED, pd, G.cls, G.pos, temb_g,
                               ln_final=ln_final)
        wgrad(gpatch, S.patches, G.pe_w, G.pe_b)
        return gpatch

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
    P = collect(conv, len(model.blocks), model.embed_dim)
    if FOLD_LN:
        _fold_cached(model, named).attach(P)
    return P


def _fold_cached(model, named: Dict[str, torch.Tensor]) -> LnFold:
    """LnFold of the given fp32 parameters, recomputed when any input changes version."""
    depth = len(model.blocks)
    key = tuple((named[n].data_ptr(), named[n]._version, named[n].device) for n in LnFold.names(depth))
    cache = model.__dict__.get("_ln_fold")
    if cache is not None and cache[0] == key:
        return cache[1]
    fold = LnFold({n: p.detach() for n, p in named.items()}, depth)
    fold.refresh()
    model.__dict__["_ln_fold"] = (key, fold)
    return fold


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
