"""DiffusionVisionTransformer — the ViT denoiser, MI355X-first.

API parity with the reference model class (`ViT_draft2drawing.py:175-329`,
duplicated in `ViT.py:158-256`):

* constructor signature and defaults (`ViT_draft2drawing.py:177-179`),
* attribute names (`num_features`, `embed_dim`, `patch_size`, `in_chans`,
  `img_size`, `total_steps`, `patch_embed.num_patches`),
* module tree / ``state_dict`` keys, shapes and ``named_parameters`` order
  (``cls_token, pos_embed, patch_embed.proj.*, time_embed.weight, blocks.*,
  norm.*, head.*`` — SURVEY §2.6), so reference ``.pkl`` checkpoints load
  with ``strict=True``,
* ``forward(x, t)`` returning an image of the input's shape (x0 / x_{t-1}
  prediction, `ViT.py:208-218`), ``prepare_tokens`` (`ViT.py:199-206`),
  the samplers (``sampler``, ``diffusion_sequence``, ``cold_sampler``,
  ``cold_diffusion_sequence``) and ``Block.forward(x, return_attention)`` /
  ``Attention.forward -> (x, attn)``.

Design (not a translation): the modules below are *parameter containers*
plus a plain-PyTorch oracle path (``forward_reference``).  On a GPU the
forward/backward run through the fused HIP kernel program in
:mod:`ddim_cold_amd.models.program` (LayerNorm, MFMA GEMMs with fused
bias/GELU/dropout/DropPath/residual epilogues, fused attention, patch-embed
with cls/pos/time fusion and an unpatchifying head), wrapped in one autograd
Function so ``loss.backward()`` still works for library users.
"""
from __future__ import annotations

import math
import os
from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

__all__ = [
    "trunc_normal_",
    "drop_path",
    "DropPath",
    "Mlp",
    "Attention",
    "Block",
    "PatchEmbed",
    "positionalencoding1d",
    "sinusoidal_timestep_embedding",
    "DiffusionVisionTransformer",
]


def trunc_normal_(tensor: torch.Tensor, mean: float = 0.0, std: float = 1.0,
                  a: float = -2.0, b: float = 2.0) -> torch.Tensor:
    """Truncated-normal init (`ViT.py:12-50` semantics: inverse-CDF sampling).

    Delegates to ``torch.nn.init.trunc_normal_`` which implements the same
    inverse-CDF method; kept as a module-level name for API parity.
    """
    return nn.init.trunc_normal_(tensor, mean=mean, std=std, a=a, b=b)


def drop_path(x: torch.Tensor, drop_prob: float = 0.0, training: bool = False) -> torch.Tensor:
    """Per-sample stochastic depth (`ViT.py:52-60`): keep w.p. 1-p, scale 1/(1-p)."""
    if drop_prob == 0.0 or not training:
        return x
    keep = 1.0 - drop_prob
    shape = (x.shape[0],) + (1,) * (x.ndim - 1)
    mask = torch.empty(shape, dtype=x.dtype, device=x.device).bernoulli_(keep)
    return x * (mask / keep)


class DropPath(nn.Module):
    """Stochastic depth module (`ViT.py:63-71`)."""

    def __init__(self, drop_prob: Optional[float] = None):
        super().__init__()
        self.drop_prob = float(drop_prob or 0.0)

    def forward(self, x):
        return drop_path(x, self.drop_prob, self.training)


class Mlp(nn.Module):
    """fc1 -> GELU(erf) -> Dropout -> fc2 -> Dropout (`ViT.py:74-90`)."""

    def __init__(self, in_features, hidden_features=None, out_features=None,
                 act_layer=nn.GELU, drop=0.0):
        super().__init__()
        out_features = out_features or in_features
        hidden_features = hidden_features or in_features
        self.fc1 = nn.Linear(in_features, hidden_features)
        self.act = act_layer()
        self.fc2 = nn.Linear(hidden_features, out_features)
        self.drop = nn.Dropout(drop)

    def forward(self, x):
        return self.drop(self.fc2(self.drop(self.act(self.fc1(x)))))


class Attention(nn.Module):
    """Multi-head self attention returning ``(x, attn)`` (`ViT.py:93-117`)."""

    def __init__(self, dim, num_heads=8, qkv_bias=False, qk_scale=None,
                 attn_drop=0.0, proj_drop=0.0):
        super().__init__()
        self.num_heads = num_heads
        head_dim = dim // num_heads
        self.scale = qk_scale or head_dim ** -0.5
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(dim, dim)
        self.proj_drop = nn.Dropout(proj_drop)

    def forward(self, x):
        B, N, C = x.shape
        H = self.num_heads
        qkv = self.qkv(x).view(B, N, 3, H, C // H)
        q, k, v = qkv.unbind(dim=2)  # each [B, N, H, hd]
        q, k, v = (z.transpose(1, 2) for z in (q, k, v))  # [B, H, N, hd]
        attn = torch.softmax((q @ k.transpose(-2, -1)) * self.scale, dim=-1)
        attn = self.attn_drop(attn)
        y = (attn @ v).transpose(1, 2).reshape(B, N, C)
        return self.proj_drop(self.proj(y)), attn


class Block(nn.Module):
    """Pre-norm transformer block (`ViT.py:120-138`)."""

    def __init__(self, dim, num_heads, mlp_ratio=4.0, qkv_bias=False, qk_scale=None,
                 drop=0.0, attn_drop=0.0, drop_path=0.0, act_layer=nn.GELU,
                 norm_layer=nn.LayerNorm):
        super().__init__()
        self.norm1 = norm_layer(dim)
        self.attn = Attention(dim, num_heads=num_heads, qkv_bias=qkv_bias, qk_scale=qk_scale,
                              attn_drop=attn_drop, proj_drop=drop)
        self.drop_path = DropPath(drop_path) if drop_path > 0.0 else nn.Identity()
        self.norm2 = norm_layer(dim)
        self.mlp = Mlp(in_features=dim, hidden_features=int(dim * mlp_ratio),
                       act_layer=act_layer, drop=drop)
        # kept for the fused program (drop-path probability of this block)
        self.drop_path_prob = float(drop_path)

    def forward(self, x, return_attention=False):
        y, attn = self.attn(self.norm1(x))
        if return_attention:
            return attn
        x = x + self.drop_path(y)
        return x + self.drop_path(self.mlp(self.norm2(x)))


class PatchEmbed(nn.Module):
    """Non-overlapping patch projection (`ViT.py:141-155`).

    Parameter layout identical to the reference (a ``Conv2d`` with k=s=p);
    on the GPU the projection is run as an MFMA GEMM over patch rows.
    """

    def __init__(self, img_size=(224, 224), patch_size=16, in_chans=3, embed_dim=768):
        super().__init__()
        img_size = list(img_size)
        self.img_size = img_size
        self.patch_size = patch_size
        self.num_patches = (img_size[0] // patch_size) * (img_size[1] // patch_size)
        self.proj = nn.Conv2d(in_chans, embed_dim, kernel_size=patch_size, stride=patch_size)

    def forward(self, x):
        return self.proj(x).flatten(2).transpose(1, 2)


def positionalencoding1d(d_model: int, length: int) -> torch.Tensor:
    """1-D sin/cos table ``[length, d_model]`` (`ViT_draft2drawing.py:140-156`).

    Even columns hold sin, odd columns cos, frequencies 10000^(-2i/d).
    Raises for odd ``d_model`` like the reference.
    """
    if d_model % 2 != 0:
        raise ValueError(f"Cannot use sin/cos positional encoding with odd dim (got dim={d_model})")
    pos = torch.arange(length, dtype=torch.float32).unsqueeze(1)
    inv = torch.exp(torch.arange(0, d_model, 2, dtype=torch.float32) * -(math.log(10000.0) / d_model))
    table = torch.zeros(length, d_model)
    table[:, 0::2] = torch.sin(pos * inv)
    table[:, 1::2] = torch.cos(pos * inv)
    return table


def sinusoidal_timestep_embedding(total_steps: int, dim: int) -> torch.Tensor:
    """Sinusoidal timestep table ``[total_steps, dim]`` (optional extra; the
    parity path uses the learned ``nn.Embedding`` — SURVEY §0)."""
    return positionalencoding1d(dim, total_steps)


def _fused_allowed(x: torch.Tensor) -> bool:
    if not x.is_cuda:
        return False
    if os.environ.get("DDIM_COLD_FORCE_REFERENCE", "0") == "1":
        return False
    return True


class DiffusionVisionTransformer(nn.Module):
    """ViT denoiser for DDIM / cold diffusion (`ViT_draft2drawing.py:175-238`)."""

    def __init__(self, img_size=(64, 64), patch_size=8, in_chans=3, embed_dim=256, depth=3,
                 num_heads=4, mlp_ratio=1.0, qkv_bias=True, qk_scale=None, drop_rate=0.1,
                 attn_drop_rate=0.1, drop_path_rate=0.1, norm_layer=nn.LayerNorm,
                 emb=PatchEmbed, total_steps=2000, timestep_embedding: str = "learned",
                 init_order: str = "draft2drawing", **kwargs):
        super().__init__()
        if init_order not in ("draft2drawing", "vit"):
            raise ValueError(f"init_order must be 'draft2drawing' or 'vit', got {init_order!r}")
        img_size = list(img_size)
        self.num_features = self.embed_dim = embed_dim
        self.patch_size = patch_size
        self.in_chans = in_chans
        self.img_size = img_size
        self.total_steps = total_steps
        self.num_heads = num_heads
        self.depth = depth
        self.mlp_ratio = mlp_ratio
        self.drop_rate = float(drop_rate)
        self.attn_drop_rate = float(attn_drop_rate)
        self.drop_path_rate = float(drop_path_rate)
        self.qk_scale = qk_scale
        self.timestep_embedding = timestep_embedding
        self.patch_embed = emb(img_size=img_size, patch_size=patch_size, in_chans=in_chans,
                               embed_dim=embed_dim)
        num_patches = self.patch_embed.num_patches
        # registration order mirrors the reference so named_parameters() /
        # state_dict() order is identical (own params first: cls, pos).
        self.cls_token = nn.Parameter(torch.zeros(1, 1, embed_dim))
        self.time_embed = nn.Embedding(total_steps, embed_dim)
        self.pos_embed = nn.Parameter(torch.zeros(1, num_patches + 1, embed_dim))
        # RNG draw order: the trainer's model class (ViT_draft2drawing.py:194-195, imported by
        # multi_gpu_trainer.py:6) draws pos_embed before the blocks are built; ViT.py:184 after
        # the head.  Same seed => same initial weights as the chosen reference class.
        if init_order == "draft2drawing":
            trunc_normal_(self.pos_embed, std=0.02)
        self.pos_drop = nn.Dropout(p=drop_rate)
        dpr = [float(v) for v in torch.linspace(0, drop_path_rate, depth)]
        self.blocks = nn.ModuleList([
            Block(dim=embed_dim, num_heads=num_heads, mlp_ratio=mlp_ratio, qkv_bias=qkv_bias,
                  qk_scale=qk_scale, drop=drop_rate, attn_drop=attn_drop_rate, drop_path=dpr[i],
                  norm_layer=norm_layer)
            for i in range(depth)])
        self.norm = norm_layer(embed_dim)
        self.head = nn.Linear(embed_dim, in_chans * patch_size ** 2)
        if init_order == "vit":
            trunc_normal_(self.pos_embed, std=0.02)
        trunc_normal_(self.cls_token, std=0.02)
        trunc_normal_(self.time_embed.weight, std=0.02)
        self.apply(self._init_weights)
        if timestep_embedding == "sinusoidal":
            # fixed (non-learned) table: same tensor name/shape so checkpoints stay compatible
            with torch.no_grad():
                self.time_embed.weight.copy_(sinusoidal_timestep_embedding(total_steps, embed_dim))
            self.time_embed.weight.requires_grad_(False)
        self._program = None  # lazily-built fused program (GPU)

    @staticmethod
    def _init_weights(m):
        if isinstance(m, nn.Linear):
            trunc_normal_(m.weight, std=0.02)
            if m.bias is not None:
                nn.init.constant_(m.bias, 0)
        elif isinstance(m, nn.LayerNorm):
            nn.init.constant_(m.bias, 0)
            nn.init.constant_(m.weight, 1.0)

    # ------------------------------------------------------------------ geometry
    @property
    def grid(self):
        return self.img_size[0] // self.patch_size, self.img_size[1] // self.patch_size

    @property
    def num_tokens(self) -> int:
        return self.patch_embed.num_patches + 1

    def drop_path_probs(self) -> List[float]:
        return [blk.drop_path_prob for blk in self.blocks]

    # ------------------------------------------------------------------ reference path
    def prepare_tokens(self, x, steps):
        """Patch embed + cls + pos + time embedding + pos_drop (`ViT.py:199-206`)."""
        B = x.shape[0]
        tok = self.patch_embed(x)
        tok = torch.cat((self.cls_token.expand(B, -1, -1), tok), dim=1)
        tok = tok + self.pos_embed + self.time_embed(steps).unsqueeze(1)
        return self.pos_drop(tok)

    def unpatchify(self, tok_pixels: torch.Tensor) -> torch.Tensor:
        """[B, P, p*p*C] -> [B, C, H, W] (head feature f = (a*p+b)*C + c)."""
        B = tok_pixels.shape[0]
        Hp, Wp = self.grid
        p, C = self.patch_size, self.in_chans
        img = tok_pixels.reshape(B, Hp, Wp, p, p, C).permute(0, 5, 1, 3, 2, 4)
        return img.reshape(B, C, Hp * p, Wp * p)

    def patchify(self, img: torch.Tensor) -> torch.Tensor:
        """Inverse of :meth:`unpatchify`: [B, C, H, W] -> [B, P, p*p*C]."""
        B = img.shape[0]
        Hp, Wp = self.grid
        p, C = self.patch_size, self.in_chans
        t = img.reshape(B, C, Hp, p, Wp, p).permute(0, 2, 4, 3, 5, 1)
        return t.reshape(B, Hp * Wp, p * p * C)

    def forward_reference(self, x, t):
        """Plain-PyTorch oracle forward (`ViT.py:208-218` semantics)."""
        h = self.prepare_tokens(x, t)
        for blk in self.blocks:
            h = blk(h)
        h = self.head(self.norm(h))
        return self.unpatchify(h[:, 1:, :])

    # ------------------------------------------------------------------ fused path
    def program(self):
        from .program import ViTProgram
        if self._program is None or not self._program.matches(self):
            self._program = ViTProgram.from_model(self)
        return self._program

    def forward(self, x, t):
        if _fused_allowed(x):
            from .program import fused_vit_forward
            return fused_vit_forward(self, x, t)
        return self.forward_reference(x, t)

    def get_last_selfattention(self, x, t):
        h = self.prepare_tokens(x, t)
        for i, blk in enumerate(self.blocks):
            if i < len(self.blocks) - 1:
                h = blk(h)
            else:
                return blk(h, return_attention=True)

    # ------------------------------------------------------------------ samplers
    @torch.no_grad()
    def sampler(self, device, k=10, N=128, generator=None, use_graph=True, verbose=False):
        """DDIM k-step sampler (`ViT.py:220-237`); returns CPU images in [0, 1]."""
        from ..diffusion.samplers import DDIMSampler
        return DDIMSampler(self, device, k=k, use_graph=use_graph).sample(N, generator=generator,
                                                                            verbose=verbose)

    @torch.no_grad()
    def diffusion_sequence(self, device, k=100, N=5, generator=None):
        """DDIM trajectory recorder (`ViT.py:239-256`): [x_T, x0_hat_1, ...] on CPU."""
        from ..diffusion.samplers import DDIMSampler
        return DDIMSampler(self, device, k=k, use_graph=False).sequence(N, generator=generator)

    @torch.no_grad()
    def cold_sampler(self, device, k=10, N=49, generator=None, use_graph=True):
        """Cold (de-pixelation) sampler (`ViT_draft2drawing.py:259-288`); ``k`` unused."""
        from ..diffusion.samplers import ColdSampler
        return ColdSampler(self, device, use_graph=use_graph).sample(N, generator=generator)

    @torch.no_grad()
    def cold_diffusion_sequence(self, device, N=5, generator=None):
        """Cold trajectory recorder (`ViT_draft2drawing.py:290-309`)."""
        from ..diffusion.samplers import ColdSampler
        return ColdSampler(self, device, use_graph=False).sequence(N, generator=generator)
