"""One train_worker run on the GPU (tests/test_trainer_overlap_gpu.py drives several).

The data-parallel trainer path on ONE GPU: ``force_segments`` puts the real
data-parallel step -- a 1-rank RCCL process group, the comm stream, per-bucket
counter hand-offs with the collectives pre-issued ahead of the compute-graph
replay -- under ``train_worker`` (multi_gpu_trainer.py:115-134 semantics).
With ``DDIM_COLD_FAKE_COMM=1`` every bucket's "collective" is a read-modify-write
pass over its gradient range on the comm stream: it returns correct gradients
only if it really runs after the bucket's gradients are final, so a broken
hand-off shows as a parameter mismatch against the inline layout.

    python tools/trainer_overlap_gpu.py <out.pt> [force_segments 0|1] [layout|-]
prints one JSON line (steps, ms_per_step, handoff_order, comm_choice) and saves
the final parameters to <out.pt>.
"""
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from ddim_cold_amd.config import ExperimentConfig
from ddim_cold_amd.train.trainer import Paths, train_worker


def main():
    out = sys.argv[1]
    force = len(sys.argv) > 2 and sys.argv[2] == "1"
    layout = sys.argv[3] if len(sys.argv) > 3 and sys.argv[3] != "-" else None
    steps = int(os.environ.get("OVERLAP_STEPS", "60"))
    with tempfile.TemporaryDirectory() as d:
        cfg = ExperimentConfig(initializing="init.pkl", framework="_ov", num_gpus=1, batch_size=16,
                               epoch=[0, 1], synthetic=True, synthetic_size=32 * steps, log_every=20,
                               max_steps=steps, eval_every=1, ckpt_dir=os.path.join(d, "Saved_Models"),
                               force_segments=force, comm_layout=layout, comm_autotune=False,
                               perf_log=True).validate()
        paths = Paths.make(cfg, "ov", root=d)
        # identical init weights for every run: seed-0 model saved by the trainer's rank 0
        res = train_worker(0, 1, cfg, "ov", paths)
        last = torch.load(os.path.join(paths.ckpt_dir, "lastepoch.pkl"), weights_only=True)
        torch.save({k: v for k, v in last["state_dict"].items()}, out)
    print(json.dumps({k: res[k] for k in ("steps", "ms_per_step", "handoff_order", "comm_choice", "loss_rec")}),
          flush=True)


if __name__ == "__main__":
    main()
