#!/usr/bin/env python3
"""Compatibility demo: cold de-pixelation sequence + zero-shot draft -> drawing.

Reference behaviour (ViT_draft2drawing.py:331-419): load the ViT-tiny cold
model (``Saved_Models/20220822vit_tiny_diffusion/bestloss.pkl``), write a cold
de-pixelation trajectory grid (5 samples x 7 columns), then noise a draft
image to t_start in 1599..1999 (step 50), denoise each with DDIM k=10 and
write the 1 x 10 grid ``draft2img.png``.  Here the 9 noise levels run as one
batched, hipGraph-captured img2img call.  Without the draft / checkpoint
files (not shipped) a synthetic draft / random init is used, with a warning.
"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import torch  # noqa: E402

from ddim_cold_amd.models.vit import (Attention, Block, DiffusionVisionTransformer, DropPath, Mlp,  # noqa: E402,F401
                                      PatchEmbed, drop_path, positionalencoding1d, trunc_normal_)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--ckpt", default=os.path.join(HERE, "Saved_Models", "20220822vit_tiny_diffusion", "bestloss.pkl"))
    ap.add_argument("--draft", default=os.path.join(HERE, "Saved_Models", "draft.jpg"))
    ap.add_argument("--out_dir", default=os.path.join(HERE, "Saved_Models"))
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args(argv)
    from ddim_cold_amd.data.datasets import load_image
    from ddim_cold_amd.data.synthetic import synthetic_pool
    from ddim_cold_amd.diffusion.samplers import img2img
    from ddim_cold_amd.models import build_model
    from ddim_cold_amd.train.checkpoint import load_weights
    from ddim_cold_amd.utils.images import get_next_path, save_grid, save_sequence_grid
    device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    model = build_model("vit_tiny")
    if os.path.isfile(a.ckpt):
        load_weights(model, a.ckpt, strict=True)
    else:
        print(f"warning: {a.ckpt} not found, using random-init weights", file=sys.stderr)
    model.to(device).eval()
    g = torch.Generator().manual_seed(a.seed)
    seq = model.cold_diffusion_sequence(device, N=5, generator=g)
    p1 = save_sequence_grid(seq, get_next_path(os.path.join(a.out_dir, "denoise_sequence.png")))
    if os.path.isfile(a.draft):
        draft = load_image(a.draft, model.img_size)
    else:
        print(f"warning: {a.draft} not found, using a synthetic draft", file=sys.stderr)
        draft = synthetic_pool(1, tuple(model.img_size), seed=a.seed)[0]
    starts = list(range(1599, 2000, 50))
    out = img2img(model, draft, starts, k=a.k, device=device, generator=g)
    row = torch.cat([((draft + 1) / 2).unsqueeze(0), out], dim=0)
    p2 = save_grid(row, get_next_path(os.path.join(a.out_dir, "draft2img.png")), nrow=row.shape[0])
    print(f"wrote {p1} and {p2}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
