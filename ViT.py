#!/usr/bin/env python3
"""Compatibility sampling CLI: ``python ViT.py [--sample_n 256] [--acc_k 1]``.

Reference behaviour (ViT.py:258-316): build the Oxford-Flowers model (64x64,
p=4, D=256, depth 6, 4 heads), load ``Saved_Models/OxfordFlower.pkl``, write a
DDIM trajectory grid (k=100, 6 samples) to ``denoise_sequence.png`` and a
``sample_n`` DDIM sample grid (jump ``acc_k``) to ``samples.png``.

Differences: the model runs in eval mode (the reference left
dropout on), samplers are hipGraph-captured on the GPU, ``get_next_path``
terminates, and a missing checkpoint falls back to random init with a warning
(pretrained blobs are not shipped).  Also re-exports the model API so
``from ViT import DiffusionVisionTransformer`` keeps working.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import click  # noqa: E402
import torch  # noqa: E402

from ddim_cold_amd.models.vit import (Attention, Block, DiffusionVisionTransformer, DropPath, Mlp,  # noqa: E402,F401
                                      PatchEmbed, drop_path, trunc_normal_)
from ddim_cold_amd.utils.images import get_next_path, save_grid, save_sequence_grid  # noqa: E402


@click.command()
@click.option("--sample_n", default=256, help="Number of samples you'll get.")
@click.option("--acc_k", default=1, help="Number of step jumped during sampling.")
@click.option("--ckpt", default=os.path.join(HERE, "Saved_Models", "OxfordFlower.pkl"), help="state_dict file")
@click.option("--model", "model_name", default="oxford_flower", help="named config (ddim_cold_amd.models.MODEL_CONFIGS)")
@click.option("--out_dir", default=os.path.join(HERE, "Saved_Models"))
@click.option("--seq_n", default=6)
@click.option("--seq_k", default=100)
@click.option("--seed", default=0)
def main(sample_n, acc_k, ckpt, model_name, out_dir, seq_n, seq_k, seed):
    """DDIM sampling from a DiffusionVisionTransformer checkpoint."""
    from ddim_cold_amd.models import build_model
    from ddim_cold_amd.train.checkpoint import load_weights
    device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    model = build_model(model_name, init_order="vit")  # ViT.py:184 draw order (weights are loaded anyway)
    if os.path.isfile(ckpt):
        load_weights(model, ckpt, strict=True)
    else:
        print(f"warning: {ckpt} not found, sampling from random-init weights", file=sys.stderr)
    model.to(device).eval()
    g = torch.Generator().manual_seed(seed)
    seq = model.diffusion_sequence(device, seq_k, N=seq_n, generator=g)
    p1 = save_sequence_grid(seq, get_next_path(os.path.join(out_dir, "denoise_sequence.png")))
    imgs = model.sampler(device, acc_k, sample_n, generator=g)
    p2 = save_grid(imgs, get_next_path(os.path.join(out_dir, "samples.png")), nrow=16)
    print(f"wrote {p1} and {p2}")


if __name__ == "__main__":
    main()
