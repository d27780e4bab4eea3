"""YAML experiment config — the reference schema verbatim plus optional extensions.

Reference schema (``20220822.yaml:1-15``, consumed at ``multi_gpu_trainer.py:174-210``):

============  =====================  ==========================================
key           type                   meaning
============  =====================  ==========================================
initializing  str                    init-weights file under ``Saved_Models/``
resume        str | 'none'           path of a ``lastepoch.pkl`` to resume from
AMP           bool                   mixed precision; doubles ``batch_size``
framework     str                    experiment-dir suffix
num_gpus      int                    ranks (one per GPU)
batch_size    int                    per GPU, before the AMP doubling
epoch         [start, end]           epoch range
base_lr       float                  LR per 512 images
dataStorage   [train_dir, val_dir]   image folders
image_size    [H, W]
diff_step     int                    parsed, unused by the reference (kept)
patch_size    int
embed_dim     int
depth         int
head          int                    attention heads
============  =====================  ==========================================

Derived exactly like the reference: effective per-GPU batch = batch_size x 2
if AMP (``multi_gpu_trainer.py:191-194``); lr = base_lr x batch x num_gpus / 512
(``:196``).  On MI355X "AMP" means bf16 compute with fp32 master weights
(no loss scaling needed); the batch-doubling rule is kept for parity.

Optional extension keys (defaults reproduce the reference behaviour):
``dataset`` ('cold' | 'cold_x0' | 'gaussian'), ``synthetic`` (bool: on-device
synthetic images instead of folders), ``synthetic_size``, ``seed``,
``graph`` (hipGraph capture), ``bucket_blocks`` (all-reduce bucket size in
transformer blocks), ``comm_autotune`` (data parallel on GPUs: time the bucket
layouts on the job's ranks before training and keep the fastest, state
restored; overrides ``bucket_blocks``), ``total_steps`` (DDIM T, default 2000), ``num_workers``,
``eval_every`` (epochs), ``log_every`` (steps, default 100), ``ckpt_dir``,
``timestep_embedding`` ('learned' | 'sinusoidal'), ``max_steps`` (cap per epoch,
for smoke runs), ``comm_layout`` (fixed data-parallel gradient-exchange layout
instead of ``comm_autotune``), ``force_segments`` (testing: run the data-parallel
step on a 1-rank process group), ``graph_steps`` (optimizer steps per hipGraph
replay, default 4; the batch rows come from a device table indexed by the step
counter, so one replay runs K whole steps).
"""
from __future__ import annotations

import os
from dataclasses import asdict, dataclass, field
from typing import List, Optional

import yaml


@dataclass
class ExperimentConfig:
    initializing: str = "vit_tiny.pkl"
    resume: str = "none"
    AMP: bool = True
    framework: str = "vit_tiny_diffusion"
    num_gpus: int = 1
    batch_size: int = 16
    epoch: List[int] = field(default_factory=lambda: [0, 100])
    base_lr: float = 0.005
    dataStorage: List[str] = field(default_factory=lambda: ["", ""])
    image_size: List[int] = field(default_factory=lambda: [64, 64])
    diff_step: int = 6
    patch_size: int = 8
    embed_dim: int = 384
    depth: int = 7
    head: int = 12
    # ---- extensions
    dataset: str = "cold"
    synthetic: bool = False
    synthetic_size: int = 4096
    seed: int = 42
    graph: bool = True
    bucket_blocks: int = 2
    comm_autotune: bool = True
    total_steps: int = 2000
    num_workers: int = 8
    eval_every: int = 1
    log_every: int = 100
    ckpt_dir: Optional[str] = None
    timestep_embedding: str = "learned"
    max_steps: int = 0
    backend: Optional[str] = None
    grad_accum: int = 1           # micro-batches of per_gpu_batch per optimizer step
    use_diff_step: bool = False   # True: the model's total_steps = diff_step (reference parses it but keeps 2000)
    sync_check_every: int = 0     # debug: cross-rank parameter checksum every N steps (0 = only after init)
    fault_inject_step: int = 0    # testing: raise after this many steps (after logging), to exercise resume
    fault_inject_rank: int = -1   # testing: only this rank raises (-1: every rank) -- one dead rank mid-epoch
    perf_log: bool = True         # extra '# perf' lines (img/s, device ms/step) next to the reference lines
    comm_layout: Optional[str] = None  # data parallel: '[graph-]overlap-<blocks>' | '[graph-]inline-1' (skips comm_autotune)
    force_segments: bool = False  # testing: the data-parallel step (1-rank RCCL group, comm stream) at num_gpus 1
    graph_steps: int = 4          # optimizer steps per replayed hipGraph (1: one graph per step)

    # ------------------------------------------------------------------ derived
    @property
    def per_gpu_batch(self) -> int:
        return self.batch_size * 2 if self.AMP else self.batch_size

    @property
    def lr(self) -> float:
        return self.base_lr * self.per_gpu_batch * self.num_gpus / 512

    @property
    def model_total_steps(self) -> int:
        return int(self.diff_step) if self.use_diff_step else int(self.total_steps)

    def model_kwargs(self) -> dict:
        return dict(img_size=list(self.image_size), patch_size=self.patch_size, embed_dim=self.embed_dim,
                    depth=self.depth, num_heads=self.head, total_steps=self.model_total_steps,
                    timestep_embedding=self.timestep_embedding)

    def validate(self):
        if self.grad_accum < 1:
            raise ValueError("grad_accum must be >= 1")
        if len(self.epoch) != 2 or self.epoch[0] > self.epoch[1]:
            raise ValueError(f"epoch must be [start, end], got {self.epoch}")
        if self.image_size[0] % self.patch_size or self.image_size[1] % self.patch_size:
            raise ValueError("image_size must be divisible by patch_size")
        if self.embed_dim % self.head:
            raise ValueError("embed_dim must be divisible by head")
        if self.dataset not in ("cold", "cold_x0", "gaussian"):
            raise ValueError(f"unknown dataset kind {self.dataset!r}")
        if self.dataset.startswith("cold") and self.image_size[0] != self.image_size[1]:
            raise ValueError("cold (down-sample) datasets require square images (diffusion_loader.py:74)")
        if self.comm_layout is not None:
            base = self.comm_layout[6:] if self.comm_layout.startswith("graph-") else self.comm_layout
            if not (base == "inline-1" or (base.startswith("overlap-") and base[8:].isdigit() and int(base[8:]) >= 1)):
                raise ValueError(f"unknown comm_layout {self.comm_layout!r}")
        if self.graph_steps < 1:
            raise ValueError("graph_steps must be >= 1")
        if not self.synthetic and not all(self.dataStorage):
            raise ValueError("dataStorage needs [train_dir, val_dir] unless synthetic: true")
        return self

    def to_dict(self) -> dict:
        return asdict(self)


def load_config(path: str) -> ExperimentConfig:
    with open(path) as f:
        raw = yaml.safe_load(f) or {}
    known = set(ExperimentConfig.__dataclass_fields__)
    unknown = set(raw) - known
    if unknown:
        raise ValueError(f"unknown config keys in {path}: {sorted(unknown)}")
    cfg = ExperimentConfig(**raw)
    return cfg


def find_config(exp_name: str, search_dirs=None) -> str:
    """Locate ``<ExpName>.yaml`` (reference: next to the trainer, multi_gpu_trainer.py:176)."""
    if exp_name.endswith((".yaml", ".yml")) and os.path.isfile(exp_name):
        return exp_name
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    dirs = list(search_dirs or []) + [os.getcwd(), here, os.path.join(here, "configs")]
    for d in dirs:
        p = os.path.join(d, exp_name + ".yaml")
        if os.path.isfile(p):
            return p
    raise FileNotFoundError(f"{exp_name}.yaml not found in {dirs}")
