"""All-reduce cost model for one MI355X node (8 GPUs, fully connected xGMI) and the
gradient-bucket plan derived from it.

Reference counterpart: DDP's fixed 25 MB buckets (``multi_gpu_trainer.py:88``,
``DistributedDataParallel(model)`` with default ``bucket_cap_mb``), chosen for
NVLink/NVSwitch or PCIe.  This module sizes buckets for xGMI instead.

Topology facts the model is built on
------------------------------------
* Every pair of the node's 8 GPUs has ONE direct xGMI link (7 links per GPU, ~153
  GB/s each way).  There is no switch: a job of N ranks on one node can only use the
  N-1 links among its own GPUs.
* RCCL runs one ring per link permutation ("channels"), so a ring all-reduce of S
  bytes over N ranks moves 2(N-1)/N * S per GPU over N-1 links in parallel:

      T(S) = alpha(N) + 2 (N-1)/N * S / ((N-1) * link * eff) = alpha(N) + 2 S / (N * link * eff)

  The bandwidth term therefore SHRINKS with N (more links), and N = 2 (one link)
  is the most expensive configuration per byte: 4x the N = 8 cost.
* alpha(N) = launch + 2 (N-1) ring steps of a few microseconds each (kernel-side
  flag hand-offs over xGMI).

The constants are assumptions until measured: :func:`fit_allreduce` fits (alpha,
bus bandwidth) to all-reduce times measured on the job's own ranks
(:meth:`ddim_cold_amd.train.engine.TrainEngine.probe_allreduce`), and
``bench.py`` reports that fit at N > 1.

Bucket plan
-----------
:func:`simulate_step` replays the backward's bucket hand-offs against one serial
comm queue: bucket k's gradients are final after its blocks' backward plus its
weight-gradient launch; its all-reduce starts when both the gradients and the
previous collective are done; the optimizer waits for the last one.  The exposed
time is what the step pays over the single-process step.  :func:`plan_buckets`
evaluates every bucket size (in blocks) and returns them cheapest first;
``TrainEngine.autotune_comm`` then MEASURES the model's pick against the inline
layout on the real ranks (the model orders candidates, the clock decides).
"""
from __future__ import annotations

import dataclasses
import math
from typing import Dict, List, Optional, Sequence, Tuple

LINK_GBS = 153.0  # one xGMI link, each direction (MI355X)
LINKS_PER_GPU = 7


@dataclasses.dataclass(frozen=True)
class AllReduceModel:
    """T(S) = alpha_us + S / busbw-equivalent, see the module docstring."""
    world: int
    alpha_us: float
    algbw_gbs: float  # S / (T - alpha): effective algorithm bandwidth, GB/s

    def time_us(self, nbytes: float) -> float:
        if self.world <= 1 or nbytes <= 0:
            return 0.0
        return self.alpha_us + nbytes / (self.algbw_gbs * 1e3)

    @property
    def busbw_gbs(self) -> float:
        """nccl-tests' bus bandwidth: algbw * 2 (N-1) / N."""
        return self.algbw_gbs * 2 * (self.world - 1) / self.world


def xgmi_ring_model(world: int, link_gbs: float = LINK_GBS, eff: float = 0.7, launch_us: float = 8.0,
                    step_us: float = 1.5) -> AllReduceModel:
    """A-priori ring model on a fully connected xGMI node (assumed constants:
    ``eff`` = fraction of link bandwidth a ring channel sustains, ``step_us`` per
    ring step).  algbw = N * link * eff / 2 (N-1 rings in parallel)."""
    if world < 1 or world > LINKS_PER_GPU + 1:
        raise ValueError(f"one node has 1..{LINKS_PER_GPU + 1} GPUs, got {world}")
    if world == 1:
        return AllReduceModel(1, 0.0, math.inf)
    return AllReduceModel(world, launch_us + 2 * (world - 1) * step_us, world * link_gbs * eff / 2)


def fit_allreduce(world: int, sizes: Sequence[float], times_us: Sequence[float]) -> AllReduceModel:
    """Least-squares fit of T = alpha + S / algbw to measured all-reduce times
    (bytes, microseconds).  alpha is clamped at >= 0; with one size the whole time
    is attributed to bandwidth."""
    if len(sizes) != len(times_us) or not sizes:
        raise ValueError("sizes and times must be non-empty and of equal length")
    n = len(sizes)
    if n == 1:
        return AllReduceModel(world, 0.0, sizes[0] / max(times_us[0], 1e-9) / 1e3)
    mx = sum(sizes) / n
    my = sum(times_us) / n
    sxx = sum((x - mx) ** 2 for x in sizes)
    sxy = sum((x - mx) * (y - my) for x, y in zip(sizes, times_us))
    slope = sxy / sxx if sxx > 0 else 0.0
    alpha = my - slope * mx
    if alpha < 0 or slope <= 0:  # noisy small sizes: bandwidth-only fit through the largest
        alpha = 0.0
        i = max(range(n), key=lambda j: sizes[j])
        slope = max(times_us[i], 1e-9) / sizes[i]
    return AllReduceModel(world, alpha, 1.0 / slope / 1e3)


@dataclasses.dataclass
class StepProfile:
    """Single-process step timing + gradient sizes, backward order (last block first).

    ``block_bwd_us``: input-gradient backward of one block (its weight gradients are
    deferred to the bucket's launch); ``block_wgrad_us``: that block's share of the
    weight-gradient launch; ``bucket_overhead_us``: fixed cost of one more bucket
    (its own weight-gradient launch + counter bump + hand-off, ~13 us at one rank);
    ``tail_us``: embedding backward after block 0; ``block_bytes`` / ``embed_bytes`` /
    ``head_bytes``: gradient bytes on the wire (fp32: 4 per parameter, bf16 wire: 2)."""
    depth: int
    block_bwd_us: float
    block_wgrad_us: float
    bucket_overhead_us: float
    tail_us: float
    block_bytes: float
    embed_bytes: float
    head_bytes: float = 0.0  # the head Linear: reduced with the LAST block's bucket (first in backward order)


# ViT-tiny B=32 single-process step (profiles/graph_step_table_r3.txt): ~45 us of
# input-gradient kernels per block, 54.5 us for the step's weight-gradient GEMMs
# (7.8 us per block), 9.4 us embedding backward; ~13 us per extra bucket
# (profiles/dp/bucket_overhead_r3.txt: 1-rank RCCL step with 2 / 3 / 4 / 8 buckets)
_TINY_BLOCK_WORK = 2080 * 887_040  # tokens x block (Linear) parameters of that measurement


def vit_step_profile(depth: int, dim: int, hidden: int, batch_tokens: int, other_params: int,
                     wire_bytes: int = 4, block_bwd_us: float = 45.0, block_wgrad_us: float = 7.8,
                     tail_us: float = 9.4, bucket_overhead_us: float = 13.0) -> StepProfile:
    """StepProfile from the model shape: the measured ViT-tiny constants, scaled by
    GEMM work (tokens x block parameters) above the per-block launch floor.  A
    block's gradient bytes are its four Linears only: the engine's arena keeps every
    LayerNorm next to the embeddings, i.e. in the last bucket (``other_params``)."""
    block_params = 3 * dim * dim + 3 * dim + dim * dim + dim + 2 * dim * hidden + hidden + dim
    r = max(1.0, batch_tokens * block_params / _TINY_BLOCK_WORK)
    return StepProfile(depth=depth, block_bwd_us=block_bwd_us * r, block_wgrad_us=block_wgrad_us * r,
                       bucket_overhead_us=bucket_overhead_us, tail_us=tail_us * r,
                       block_bytes=float(block_params * wire_bytes), embed_bytes=float(other_params * wire_bytes))


def bucket_plan(prof: StepProfile, bucket_blocks: int, embed_bucket: bool = True) -> List[Tuple[int, float]]:
    """(blocks, wire bytes) per bucket in backward order -- the layout
    ``TrainEngine._build_buckets`` makes: ``bucket_blocks`` blocks per bucket from
    the last block down (the head with the first of them), the embeddings + every
    LayerNorm (``embed_bytes``) in a last
    bucket of their own when ``embed_bucket`` else with block 0's bucket."""
    out = []
    left = prof.depth
    while left > 0:
        k = min(bucket_blocks, left)
        left -= k
        out.append([k, k * prof.block_bytes + (prof.head_bytes if not out else 0.0)])
    if embed_bucket:
        out.append([0, prof.embed_bytes])
    else:
        out[-1][1] += prof.embed_bytes
    return [(k, b) for k, b in out]


def simulate_step(prof: StepProfile, model: AllReduceModel, bucket_blocks: int, embed_bucket: bool = True,
                  inline: bool = False) -> Dict[str, float]:
    """Exposed communication time of one step (us over the single-process step).

    inline: one all-reduce of every gradient after the backward (no overlap, no
    bucket overheads).  Otherwise buckets of ``bucket_blocks`` blocks in backward
    order, the embeddings (+ LayerNorms) in their own last bucket when
    ``embed_bucket``, else with block 0's bucket."""
    L = prof.depth
    total = L * prof.block_bytes + prof.embed_bytes + prof.head_bytes
    bwd_end = L * (prof.block_bwd_us + prof.block_wgrad_us) + prof.tail_us
    if inline or model.world <= 1:
        comm = model.time_us(total)
        return {"exposed_us": comm, "comm_us": comm, "buckets": 1, "bwd_us": bwd_end}
    t = 0.0
    q = 0.0  # comm queue free at
    comm_sum = 0.0
    sizes = bucket_plan(prof, bucket_blocks, embed_bucket)
    for j, (k, nbytes) in enumerate(sizes):
        t += k * (prof.block_bwd_us + prof.block_wgrad_us) + prof.bucket_overhead_us
        if j == len(sizes) - 1:
            t += prof.tail_us  # the embedding backward precedes the last bucket
        c = model.time_us(nbytes)
        q = max(q, t) + c
        comm_sum += c
    nb = len(sizes)
    # the step's own backward grew by the bucket launches; the optimizer waits for q
    exposed = max(q, t) - bwd_end
    return {"exposed_us": exposed, "comm_us": comm_sum, "buckets": nb, "bwd_us": bwd_end}


def plan_buckets(prof: StepProfile, model: AllReduceModel,
                 choices: Optional[Sequence[int]] = None) -> List[Tuple[str, int, bool, bool, float]]:
    """Every layout, cheapest predicted first: ``(name, bucket_blocks, embed_bucket,
    inline, exposed_us)`` -- the same tuple shape as ``TrainEngine.COMM_LAYOUTS`` plus
    the prediction."""
    out = []
    for bb in (choices or range(1, prof.depth + 1)):
        r = simulate_step(prof, model, bb, embed_bucket=True)
        out.append((f"overlap-{bb}", bb, True, False, r["exposed_us"]))
    r = simulate_step(prof, model, 1, inline=True)
    out.append(("inline-1", 1 << 16, False, True, r["exposed_us"]))
    out.sort(key=lambda x: x[4])
    return out


def describe(prof: StepProfile, worlds: Sequence[int] = (2, 4, 8), **model_kw) -> str:
    """Markdown table of the a-priori model over world sizes (for profiles/)."""
    lines = ["| N | algbw GB/s | alpha us | all-reduce of all grads us | best layout | exposed us | "
             "inline exposed us |", "|---:|---:|---:|---:|---|---:|---:|"]
    total = prof.depth * prof.block_bytes + prof.embed_bytes + prof.head_bytes
    for n in worlds:
        m = xgmi_ring_model(n, **model_kw)
        plan = plan_buckets(prof, m)
        inline = [p for p in plan if p[0] == "inline-1"][0]
        lines.append(f"| {n} | {m.algbw_gbs:.0f} | {m.alpha_us:.1f} | {m.time_us(total):.1f} | {plan[0][0]} | "
                     f"{plan[0][4]:.1f} | {inline[4]:.1f} |")
    return "\n".join(lines)
