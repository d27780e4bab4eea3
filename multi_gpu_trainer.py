#!/usr/bin/env python3
"""Compatibility entry point: ``python multi_gpu_trainer.py <ExpName>``.

Same contract as the reference (multi_gpu_trainer.py:167-219): reads
``<ExpName>.yaml`` (next to this file, in ``configs/`` or the CWD), derives the
per-GPU batch (x2 for AMP) and the LR (base_lr * batch * num_gpus / 512),
creates ``Saved_Models/<ExpName><framework>/`` with a copy of the YAML and
``train.log``, and trains ``num_gpus`` ranks (spawned here, or one rank per
process under ``torchrun``), on the MI355X engine.

The reference module's library functions are importable from here with their
signatures (``ddim_cold_amd/train/compat.py``): ``printLog(string, fileName)``,
``init_process_group(world_size, rank)``, ``evaluate(model, dataloader, device)``
and the rank worker ``main(rank, world_size, initializing, amp, batch_size,
epoch_num, lr, resume, datadir, SavedDir, log, CheckpointDir, image_size,
diff_step, patch_size, embed_dim, depth, head)``; the command line is :func:`cli`.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from ddim_cold_amd.train.compat import evaluate, init_process_group, main, printLog  # noqa: E402,F401


def cli(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("exp_name", help="experiment name: <ExpName>.yaml")
    ap.add_argument("--root", default=os.path.dirname(os.path.abspath(__file__)),
                    help="directory holding Saved_Models/ (reference: the script directory)")
    ap.add_argument("--backend", default=None, help="nccl (RCCL, default on GPU) | gloo")
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args(argv)
    from ddim_cold_amd.config import find_config, load_config
    from ddim_cold_amd.train.trainer import Paths, launch
    path = find_config(a.exp_name)
    cfg = load_config(path).validate()
    exp = os.path.splitext(os.path.basename(a.exp_name))[0]
    paths = Paths.make(cfg, exp, root=a.root, config_path=path)
    res = launch(cfg, exp, paths, backend=a.backend)
    if res:
        print({k: v for k, v in res.items() if k != "history"})
    return 0


if __name__ == "__main__":
    sys.exit(cli())
