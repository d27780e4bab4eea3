"""Named model configurations.

* ``vit_tiny``      — the yaml experiment config (20220822.yaml:10-15): 64x64, p=8,
                      D=384, depth 7, 12 heads, mlp_ratio 1 (the training benchmark).
* ``oxford_flower`` — the sampling CLI config (ViT.py:277): 64x64, p=4, D=256, depth 6, 4 heads.
* ``mini_imagenet`` — ViT.py:274 (commented alternative): same shape as vit_tiny.
* ``vit_small_200`` — high-resolution path (200x200). The reference ships only a
                      missing checkpoint for it (README.md:29, .MISSING_LARGE_BLOBS); the
                      architecture is OUR documented choice: p=8, D=384,
                      depth 12, 6 heads (hd 64), 626 tokens.
"""
from __future__ import annotations

from .vit import DiffusionVisionTransformer

MODEL_CONFIGS = {
    "vit_tiny": dict(img_size=[64, 64], patch_size=8, embed_dim=384, depth=7, num_heads=12, total_steps=2000),
    "oxford_flower": dict(img_size=[64, 64], patch_size=4, embed_dim=256, depth=6, num_heads=4, total_steps=2000),
    "mini_imagenet": dict(img_size=[64, 64], patch_size=8, embed_dim=384, depth=7, num_heads=12, total_steps=2000),
    "vit_small_200": dict(img_size=[200, 200], patch_size=8, embed_dim=384, depth=12, num_heads=6,
                          total_steps=2000),
}


def build_model(name: str, **overrides) -> DiffusionVisionTransformer:
    cfg = dict(MODEL_CONFIGS[name])
    cfg.update(overrides)
    return DiffusionVisionTransformer(**cfg)
