#!/usr/bin/env python3
"""Visualise the cold (pixelation) training pairs (x_t, x_{t-1}) for t = 1..log2(W).

The reference's ``diffusion_loader.py:141-154`` demo, headless: writes one grid
PNG (row t: x_t | x_{t-1}) instead of opening matplotlib windows.

    python tools/show_cold_pairs.py --folder data/OxfordFlowers/train --size 64 --out pairs.png
    python tools/show_cold_pairs.py --synthetic --out pairs.png
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from ddim_cold_amd.data.datasets import ColdDownSampleDataset  # noqa: E402
from ddim_cold_amd.data.synthetic import synthetic_pool  # noqa: E402
from ddim_cold_amd.ops import reference as ref  # noqa: E402
from ddim_cold_amd.utils.images import save_grid  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--folder", default=None)
    ap.add_argument("--synthetic", action="store_true")
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--index", type=int, default=0)
    ap.add_argument("--out", default="cold_pairs.png")
    a = ap.parse_args(argv)
    if a.folder and not a.synthetic:
        ds = ColdDownSampleDataset(a.folder, [a.size, a.size])
        pairs = [ds.__getitem__(a.index, t)[:2] for t in range(1, ds.max_step + 1)]
    else:
        img = synthetic_pool(a.index + 1, (a.size, a.size))[a.index]
        steps = int(torch.log2(torch.tensor(float(a.size))).item())
        pairs = [(ref.pixelate(img[None], 2 ** t)[0], ref.pixelate(img[None], 2 ** (t - 1))[0])
                 for t in range(1, steps + 1)]
    imgs = torch.stack([im for p in pairs for im in p])
    save_grid((imgs + 1) / 2, a.out, nrow=2)
    print(f"wrote {a.out} ({len(pairs)} pairs)")


if __name__ == "__main__":
    main()
