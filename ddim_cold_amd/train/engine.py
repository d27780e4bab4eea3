"""TrainEngine — the MI355X training step runtime.

One training step of the reference (multi_gpu_trainer.py:115-134:
autocast forward, smooth-L1, backward with DDP all-reduce, unscale, clip 1.0,
AdamW step, cosine LR step, zero_grad) re-designed for a latency-bound
7 M-parameter model on MI355X:

* **Flat arenas.**  All parameters live in one fp32 arena (``nn.Parameter.data``
  are views), gradients in a second (``param.grad`` are views), Adam moments
  in two more, plus a bf16 shadow of the parameters that the MFMA GEMMs read.
  Every param offset is 256-B aligned.  All-reduce buckets are contiguous arena
  ranges: no pack/unpack kernels.
* **Fused optimizer.**  3 launches per step (global grad-norm, AdamW + clip +
  cosine LR + bf16 shadow refresh + grad zeroing, counter bump); the LR /
  Adam step / RNG step live in device memory so the step is graph-replayable.
* **Deferred weight gradients.**  Single process: every weight-gradient GEMM
  of the step is ONE launch after the embedding backward
  (``ops.linear_wgrad_multi``, 1,548 64x64 tiles, no token split, no atomics).
  Data parallel: one such launch per gradient bucket, so each bucket's
  all-reduce can start while the remaining blocks run backward.  (Issuing them
  on a side stream measured slower: 28.2k vs 33.1k img/s.)
* **hipGraphs per step, bucketed RCCL all-reduce between them.**  Gradient
  buckets are contiguous arena ranges closed at transformer-block boundaries
  of the backward; as soon as a bucket's gradients are final its
  ``all_reduce`` (RCCL over xGMI via ``torch.distributed`` 'nccl') runs on
  a communication stream, so it overlaps the backward of the remaining
  blocks, and the optimizer waits on that stream.  Data parallel default
  (``comm_events``): forward + backward is ONE linear graph that bumps a
  per-bucket counter at every bucket boundary (a 1-lane kernel node), the
  optimizer a second; each bucket's collective waits on the comm stream
  behind a bounded polling kernel for its counter, queued ahead of the
  compute replay (a comm branch inside the graph costs ~30 us per fork on
  MI355X; event-record nodes delayed the comm work to the end of the graph).  ``autotune_comm()`` picks the bucket layout (or one
  inline all-reduce) by measuring on the job's own ranks.  Alternatives:
  collectives captured into the step graph (``graph_comm``) or
  ``n_buckets + 1`` graph segments with host-issued collectives in between.
  Buckets default to ~2 blocks (~7 MB fp32 for ViT-tiny): few enough
  collectives for the per-call latency of 7-link point-to-point xGMI rings,
  large enough to overlap.  Inactive time-embedding rows are not reduced.
"""
from __future__ import annotations

import math
import copy
import os
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from .. import ops
from ..models import program as _program
from ..models.program import LnFold, ModelTensors, ViTProgram, collect, is_matrix_param

ALIGN = 64  # elements (256 B fp32)
# Step graphs are captured in thread-local mode: other threads' HIP calls during a
# capture (ProcessGroupNCCL's watchdog polling the events of eager collectives)
# neither invalidate the capture nor fail in that thread.  In the default global
# mode a watchdog poll inside the capture window was seen on MI355X to invalidate
# the capture (fallback to segments) and abort the process from the watchdog.
CAPTURE_MODE = "thread_local"
# event-split data parallel with counter hand-offs: queue the comm stream's work
# ahead of the compute-graph replay (DDIM_COLD_PREISSUE=0: behind it)
PREISSUE = os.environ.get("DDIM_COLD_PREISSUE", "1") != "0"
# the LayerNorm dgamma/dbeta replica finalize rides in the embedding-backward launch
# (False: a separate replica_reduce_ launch; tests compare the two)
FUSE_LN_FINAL = True
# single process: the grad-norm partials come from the weight-gradient launch's
# epilogues (ops.linear_wgrad_multi sq=) instead of a separate sqnorm pass over the
# arena (False: the sqnorm kernel; tests compare the two)
FUSE_SQNORM = True
# with FUSE_SQNORM: no embedding-backward launch -- the last LayerNorm backward writes
# the patch-row gradient, and the cls / pos / time-embedding gradients and the
# LayerNorm finalize run as extra workgroups of the weight-gradient launch
# (csrc/embed_parts.h; False: embed_bwd as its own launch; tests compare the two)
FUSE_EMBED_WGRAD = True
# models of at least this many tokens per sample (vit_small_200: 626) keep transposed bf16
# shadows of the QKV / proj / fc1 / fc2 weights, re-transposed after every optimizer step, so
# their input-gradient GEMMs run on the k-contiguous operand path
# (tools/ub_dgrad_layout.py: QKV 31.7 -> 25.5 us, K = 384 15.0 -> 13.5 us at M = 20,032;
# ViT-tiny's M = 2,080 gains ~0.5 us per GEMM, less than the transpose launch costs)
TRANSPOSED_DGRAD_MIN_TOKENS = 512


class TransposedShadows:
    """Transposed copies ([in][out], bf16) of the blocks' QKV, proj, fc1 and fc2 weight
    shadows in one arena; :meth:`refresh` re-transposes all of them in one launch (after
    every optimizer step, inside the step graph), :meth:`attach` sets ``qkv_wt`` /
    ``proj_wt`` / ``fc1_wt`` / ``fc2_wt`` on the program's block tensors (fc2: the
    input gradient through GELU)."""

    KINDS = ("qkv", "proj", "fc1", "fc2")

    def __init__(self, P: ModelTensors):
        self.src = []
        for bp in P.blocks:
            self.src += [getattr(bp, k + "_w") for k in self.KINDS]
        n = sum(w.numel() for w in self.src)
        self.arena = torch.empty(n, dtype=torch.bfloat16, device=self.src[0].device)
        self.dst, o = [], 0
        for w in self.src:
            self.dst.append(self.arena[o:o + w.numel()].view(w.shape[1], w.shape[0]))
            o += w.numel()

    def refresh(self):
        ops.transpose_bf16_(self.src, self.dst)

    def attach(self, P: ModelTensors) -> ModelTensors:
        for i, bp in enumerate(P.blocks):
            for j, k in enumerate(self.KINDS):
                setattr(bp, k + "_wt", self.dst[len(self.KINDS) * i + j])
        return P


@dataclass
class EngineConfig:
    lr: float = 3.125e-4
    weight_decay: float = 0.05
    betas: Tuple[float, float] = (0.9, 0.999)
    eps: float = 1e-8
    max_grad_norm: float = 1.0
    t_max: int = 0            # cosine annealing period in optimizer steps (0: constant LR)
    eta_min: float = 0.0
    use_graph: bool = True
    graph_warmup: int = 3     # eager steps before capture
    bucket_blocks: int = 2    # transformer blocks per all-reduce bucket
    # the embedding gradients (cls / pos / patch-embed / time-embed, final only
    # after the embedding backward) get their own small last bucket, so block 0's
    # all-reduce overlaps the embedding backward and only ~0.4 MB (ViT-tiny) is
    # exposed before the optimizer
    embed_bucket: bool = True
    seed: int = 42
    loss_beta: float = 1.0
    ema_decay: float = 0.99
    ema_init: float = 5.0     # multi_gpu_trainer.py:52 (loss_rec = 5.0)
    force_segments: bool = False  # segmented capture + collectives even at world size 1 (testing)
    # rows of time_embed that can receive gradient (t < temb_rows for every sample);
    # the rest are all-zero on every rank and are left out of the all-reduce.
    # Cold diffusion draws t in 1..log2(W) (7 rows), so for ViT-tiny this drops
    # 3.1 MB of the 28.7 MB gradient all-reduce.  None: all rows.
    temb_rows: Optional[int] = None
    # data parallel with t drawn from the whole table (Gaussian diffusion, temb_rows
    # None): only the <= world x batch rows indexed by this step's timesteps carry
    # gradient, so the time_embed gradient is exchanged as all-gathered (t, row)
    # pairs (49 KB per rank for ViT-tiny at batch 32) instead of all-reducing the
    # dense [2000, 384] table (3.1 MB).  SURVEY.md §5.8 option 4.
    temb_sparse: bool = True
    # capture the bucketed all-reduces INTO the step's hipGraph (RCCL kernels on a
    # comm-stream branch joined before the optimizer) instead of replaying one
    # graph segment per bucket with host-issued collectives in between.
    # Measured on one MI355X with a 1-rank RCCL group: 0.998 ms/step captured vs
    # 1.125 segmented (each extra graph launch + stream join costs ~30 us).
    # Falls back to segments if the capture raises.
    graph_comm: bool = True
    # data parallel, the default capture: the step's compute as TWO linear graphs
    # (forward + backward, then optimizer) whose only cross-stream edges are
    # external event-record nodes at the bucket boundaries; the collectives are
    # issued by the host on the comm stream (eager RCCL, nothing of it captured),
    # each waiting on its bucket's event.  A graph with a comm-stream branch
    # (graph_comm) costs ~30-35 us per fork on MI355X -- measured on one GPU with a
    # 1-element kernel on a side stream at each of the 5 bucket boundaries: 0.818 ->
    # 1.013 ms/step -- and with one elementwise pass per bucket on the comm stream
    # (standing in for the collective) the event-split step runs at 0.937 vs 1.072
    # captured.  False: graph_comm / segments.
    comm_events: bool = True
    # data parallel: issue the collectives on the compute stream (no comm stream, no
    # overlap; with comm_events, host-issued between the two step graphs).  With one
    # bucket this is the single-process step + one all-reduce of the whole arena;
    # autotune_comm() measures it against the overlapped layouts on the real ranks.
    comm_inline: bool = False
    # micro-batches per optimizer step (batch_fn is called grad_accum times per
    # step; gradients accumulate in the arena, averaged in the optimizer; the
    # all-reduce runs once, after the last micro-batch's backward)
    grad_accum: int = 1
    # gradient all-reduce wire format: "fp32" (reference DDP semantics) or "bf16"
    # (halves the xGMI bytes; the sum is accumulated in bf16 by RCCL)
    grad_wire: str = "fp32"
    # who issues the gradient collectives: "torch" (torch.distributed 'nccl' =
    # RCCL through ProcessGroupNCCL) or "native" (csrc/comm.cpp: our own
    # ncclComm_t, collectives enqueued directly on the comm stream, bf16 wire
    # pack/unpack as two fused kernels).  torch.distributed stays the control
    # plane (rendezvous, barriers, metrics) either way.
    # "auto" (default): native when it initialises and verifies on every rank of the
    # default group (GPU), else torch
    comm: str = "auto"
    # a batch source with ``fused_spec()`` (data.synthetic.ColdBatcher) has its draw
    # fused into the patch-embedding launch (ops.patch_embed_cold_fwd: the patch rows
    # pixelated straight from the pool, x_t never materialised): one launch fewer
    # per step, identical values.
    fuse_batch: bool = True
    # optimizer steps per hipGraph replay for train_steps(n) (one graph holding K
    # complete steps, every counter on the device): the inter-replay dispatch gap
    # (~8 us before each step's first kernel in the graph-mode trace) is paid once
    # per K steps.  train_step() keeps replaying the one-step graph.
    graph_steps: int = 1


def _align(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


class TrainEngine:
    def __init__(self, model, cfg: EngineConfig = EngineConfig(), device=None, process_group=None):
        self.cfg = cfg
        self.model = model
        self.device = torch.device(device) if device is not None else next(model.parameters()).device
        model.to(self.device)
        self.prog = ViTProgram.from_model(model)
        self.pg = process_group
        self.dist_on = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(process_group) if self.dist_on else 1
        self.rank = dist.get_rank(process_group) if self.dist_on else 0
        self.segmented = self.world > 1 or cfg.force_segments
        self.is_cuda = self.device.type == "cuda"
        self._build_arenas()
        dev = self.device
        self.rng = torch.tensor([cfg.seed, 0], dtype=torch.int64, device=dev)
        self.step_ctr = torch.zeros(2, dtype=torch.int64, device=dev)  # {adam step, scheduler step}
        b1, b2 = cfg.betas
        self.hyper = torch.tensor([cfg.lr, b1, b2, cfg.eps, cfg.weight_decay, cfg.max_grad_norm,
                                   float(cfg.t_max), cfg.eta_min], dtype=torch.float32, device=dev)
        # grad-norm partials (sqnorm, or the fused weight-gradient launch: one per 64x64
        # output tile + tail workgroups; the 2-D parameter count bounds the tiles)
        tiles = sum(-(-p.shape[0] // 64) * -(-(p[0].numel()) // 64) for p in model.parameters() if p.dim() >= 2)
        self._sq_tiles = tiles
        self.sqnorm = torch.zeros(ops.sq_parts_size(tiles), dtype=torch.float32, device=dev)
        self.loss_last = torch.zeros(1, dtype=torch.float32, device=dev)
        self.loss_ema = torch.full((1,), cfg.ema_init, dtype=torch.float32, device=dev)
        # the comm stream is created once and kept across set_comm_layout() (a stream
        # created later could land on a hardware queue another stream already holds)
        self._comm_obj = self._comm_stream() if (self.is_cuda and self.segmented) else None
        self.comm = None if cfg.comm_inline else self._comm_obj
        self.handoff_order: Optional[str] = None  # event-split step: "pre-issued" / "post-replay"
        self.comm_choice: Optional[str] = None  # autotune_comm() winner
        self.comm_times: Dict[str, float] = {}
        if cfg.comm not in ("torch", "native", "auto"):
            raise ValueError(f"comm must be 'torch', 'native' or 'auto', got {cfg.comm!r}")
        self.ncomm = None
        self.native_error: Optional[str] = None  # why comm='auto' fell back to torch.distributed
        self.comm_fallback: Optional[str] = None  # autotune_comm: why no layout ran (eager inline fallback)
        default_pg = process_group is None or process_group is dist.group.WORLD
        if cfg.comm == "native" and self.dist_on and self.is_cuda:
            if not default_pg:
                raise ValueError("comm='native' spans the default process group only")
            from ..parallel.comm import NativeComm
            self.ncomm = NativeComm(dev)
        elif cfg.comm == "auto" and self.dist_on and self.is_cuda and default_pg:
            self.ncomm = self._try_native(dev)
        self.comm_backend = "native" if self.ncomm is not None else "torch"
        self._graphs: Optional[List[torch.cuda.CUDAGraph]] = None
        self._graph_comm_failed = False  # captured collectives refused -> per-bucket segments
        self._multi = None  # (K-step graph, K) for train_steps
        self._eager_steps = 0
        self.batch_fn: Optional[Callable] = None
        self._static = None
        self.steps_done = 0
        if self.world > 1:
            if self.ncomm is not None:
                self.ncomm.broadcast_(self.flat_p, 0)
            else:
                dist.broadcast(self.flat_p, src=0, group=self.pg)
            self._refresh_shadow()
        model._engine = self

    def _comm_stream(self):
        """The collectives' stream, high priority.  HIP keeps a separate pool of hardware queues per priority, so a
        high-priority comm stream can never share an in-order hardware queue with the
        normal-priority compute stream -- with GPU_MAX_HW_QUEUES=4 normal-priority
        streams beyond four do share queues round-robin, and a comm-stream wait
        queued ahead of the compute graph on a SHARED queue would block that graph
        (see :meth:`_preissue_ok`)."""
        return torch.cuda.Stream(device=self.device, priority=-1)

    def _preissue_ok(self) -> bool:
        """Queue the comm stream's counter waits + collectives AHEAD of the compute
        graph replay only when that cannot deadlock-until-timeout: RCCL issue never
        blocks the host, and the comm stream has a different priority from the
        compute stream, i.e. its own hardware queue.  Otherwise the host issues them
        after the replay (same overlap, ~2-3 us later start per bucket)."""
        if not (PREISSUE and self.comm is not None and self._comm_host_async()):
            return False
        return self.comm.priority != torch.cuda.current_stream(self.device).priority

    def _try_native(self, dev):
        """comm='auto': our own RCCL communicator if it comes up and sums correctly on
        EVERY rank (agreed through the torch process group), else torch.distributed.
        Its collectives are enqueued straight on the issuing stream; ProcessGroupNCCL
        runs each on its internal stream behind an event round trip each way (1-rank
        inline step: 0.849 vs 0.866 ms)."""
        import warnings
        from ..parallel.watchdog import phase
        phase("native-comm:check")
        # every rank must be able to enter ncclCommInitRank before any does: the init
        # blocks until all ranks have joined, so a rank that fails BEFORE it (no
        # extension, no comm ops) would leave the others hanging there
        ready = 1
        try:
            from ..ops import _ext
            _ext.load(raise_on_error=True)
            ready = int(hasattr(torch.ops.ddim_cold, "comm_init"))
        except Exception as e:  # pragma: no cover - depends on the build
            warnings.warn(f"native RCCL communicator unavailable ({e!r})")
            ready = 0
        flag = torch.tensor([ready], dtype=torch.int32, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.pg)
        if int(flag.item()) != 1:
            return None
        nc, ok = None, 1
        phase("native-comm:init")
        try:
            from ..parallel.comm import NativeComm
            nc = NativeComm(dev)
            phase("native-comm:verify", ranks=nc.info()[0])
            x = torch.full((4 * self.world + 3,), float(self.rank + 1), device=dev)
            nc.all_reduce_(x)
            torch.cuda.synchronize(dev)
            ok = int(bool((x == self.world * (self.world + 1) / 2).all()))
            if not ok:
                self.native_error = "verification sum mismatch"
        except Exception as e:  # noqa: BLE001 - any failure falls back to torch.distributed
            warnings.warn(f"native RCCL communicator unavailable ({e!r}); using torch.distributed")
            self.native_error = repr(e)[:300]
            ok = 0
        flag = torch.tensor([ok], dtype=torch.int32, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.pg)
        if int(flag.item()) == 1:
            phase("native-comm:ready", ranks=self.world)
            return nc
        if self.native_error is None:
            self.native_error = "failed on another rank"
        if nc is not None and nc.handle is not None:
            nc.destroy()
        phase("native-comm:fallback-torch", error=self.native_error)
        return None

    def _comm_host_async(self) -> bool:
        """True when issuing a collective never blocks the host on device progress
        (RCCL: ours or ProcessGroupNCCL).  gloo with CUDA tensors waits on the host for
        its device-to-host copy, so its collectives must not be queued ahead of the
        compute graph they wait for."""
        if self.ncomm is not None:
            return True
        try:
            return dist.get_backend(self.pg) == "nccl"
        except Exception:  # pragma: no cover
            return False

    def check_comm(self):
        """Raise ``RuntimeError`` if a comm-stream hand-off wait timed out (FlagSignal):
        that bucket's collective then ran on gradients that were not final yet, so the
        replicas may have diverged -- the run must stop (and resume from a checkpoint),
        not continue.  One host sync; call at log points, not every step."""
        sig = getattr(self, "_signal", None)
        if sig is not None:
            sig.check()

    def comm_error(self) -> bool:
        """True if a hand-off wait has timed out since the last :meth:`reset_comm_error`."""
        sig = getattr(self, "_signal", None)
        return sig is not None and sig.failed()

    def reset_comm_error(self):
        sig = getattr(self, "_signal", None)
        if sig is not None:
            sig.err.zero_()

    def attach_comm(self, comm, world: int):
        """Drive the gradient exchange through ``comm`` (the ``all_reduce_`` of a
        NativeComm-like object) as one of ``world`` data-parallel replicas without a
        process group -- e.g. two engines of one process on one device joined by a
        :class:`parallel.comm.LoopbackPair` (tests of the cross-rank hand-off).  Needs
        ``force_segments`` (the data-parallel step); the replicas must start from the
        same parameters (no broadcast here)."""
        if not (self.segmented and self.is_cuda):
            raise ValueError("attach_comm needs a GPU engine built with force_segments=True")
        if self.temb_bucket is not None and not hasattr(comm, "all_gather_"):
            raise ValueError(f"{type(comm).__name__} has no all_gather_, which this engine's sparse time-embedding "
                             "gradient exchange needs (Gaussian diffusion: temb_rows=None); build the engine "
                             "with temb_rows or temb_sparse=False")
        self.ncomm = comm
        self.world = int(world)
        self.comm_backend = type(comm).__name__
        self._graphs = None
        self._multi = None

    def close(self):
        """Release the native communicator (before the process group is destroyed)."""
        self.materialize_lazy()
        if self.ncomm is not None:
            if self.is_cuda:
                torch.cuda.synchronize(self.device)
            self.ncomm.destroy()
            self.ncomm = None

    # ------------------------------------------------------------------ arenas
    def _build_arenas(self):
        named = list(self.model.named_parameters())
        self.names = [n for n, _ in named]
        self.offsets: Dict[str, Tuple[int, int]] = {}
        # LayerNorm weight+bias are packed back to back (one [2D] range for the
        # replica finalize); every other tensor starts 256-B aligned.
        ln_prefixes = {n[: -len(".weight")] for n, p in named
                       if n.endswith(".weight") and p.dim() == 1 and (n.startswith("norm") or ".norm" in n)}
        # arena order: embeddings, then EVERY LayerNorm, then the blocks' Linear
        # weights, then the head.  The LayerNorm gradients are finalised once, in the
        # embedding-backward launch (their dgamma/dbeta replicas are only complete
        # then); placed here they fall in the last all-reduce bucket, so data
        # parallel needs no replica finalize launch per bucket either.
        # Frozen tensors (requires_grad=False, e.g. the fixed sinusoidal time table,
        # ViT_draft2drawing.py:140-156) go last, past ``train_hi``: the norm, AdamW and
        # the all-reduce buckets cover [0, train_hi) only, so a frozen tensor gets no
        # weight decay, no moments and no optimizer state (torch.optim skips a
        # parameter whose .grad is None).
        self.frozen = {n for n, p in named if not p.requires_grad}

        def group(n):
            if n in self.frozen:
                return 4
            if n.rsplit(".", 1)[0] in ln_prefixes:
                return 1
            if n.startswith("blocks."):
                return 2
            return 3 if n.startswith("head.") else 0
        layout = sorted(named, key=lambda np_: group(np_[0]))  # stable: original order within a group
        off = 0
        self.train_hi = None
        for n, p in layout:
            ln_bias = n.endswith(".bias") and n[: -len(".bias")] in ln_prefixes
            if not ln_bias:
                off = _align(off)
            if n in self.frozen and self.train_hi is None:
                self.train_hi = off
            self.offsets[n] = (off, p.numel())
            off += p.numel()
        off = _align(off)
        self.numel = off
        if self.train_hi is None:
            self.train_hi = off
        dev = self.device
        self.flat_p = torch.zeros(off, dtype=torch.float32, device=dev)
        self.flat_g = torch.zeros(off, dtype=torch.float32, device=dev)
        self.flat_m = torch.zeros(off, dtype=torch.float32, device=dev)
        self.flat_v = torch.zeros(off, dtype=torch.float32, device=dev)
        self.flat_pb = torch.zeros(off, dtype=torch.bfloat16, device=dev)
        if self.cfg.grad_wire not in ("fp32", "bf16"):
            raise ValueError(f"grad_wire must be 'fp32' or 'bf16', got {self.cfg.grad_wire!r}")
        self.flat_gw = torch.zeros(off, dtype=torch.bfloat16, device=dev) if self.cfg.grad_wire == "bf16" else None
        views_p, views_g = {}, {}
        for n, p in named:
            o, k = self.offsets[n]
            vp = self.flat_p[o:o + k].view_as(p)
            vp.copy_(p.data)
            p.data = vp
            vg = self.flat_g[o:o + k].view_as(p)
            p.grad = None if n in self.frozen else vg
            views_g[n] = vg
        # the optimizer's ranges (frozen tensors excluded)
        th = self.train_hi
        self.opt_p, self.opt_g, self.opt_m, self.opt_v, self.opt_pb = (
            t[:th] for t in (self.flat_p, self.flat_g, self.flat_m, self.flat_v, self.flat_pb))
        c = self.prog.cfg
        # LayerNorm fold: gamma-scaled bf16 weights / row sums / folded biases of
        # the QKV, fc1 and head GEMMs, recomputed from the fp32 masters after
        # every optimizer step (inside the step graph)
        # (reads the bf16 shadow the optimizer just wrote: half the bytes of the fp32 masters)
        self.lnfold = LnFold({n: p.data for n, p in named}, c.depth,
                             weights={n: self.flat_pb[o:o + k].view(p.shape)
                                      for n, p in named for o, k in [self.offsets[n]] if is_matrix_param(n)}) \
            if _program.FOLD_LN else None
        self._refresh_shadow()
        for n, p in named:
            o, k = self.offsets[n]
            views_p[n] = self.flat_pb[o:o + k].view(p.shape) if is_matrix_param(n) else p.data
        self.param_tensors: ModelTensors = collect(views_p, c.depth, c.dim)
        if self.lnfold is not None:
            self.lnfold.attach(self.param_tensors)
        self.wt = None
        if self.is_cuda and c.tokens >= TRANSPOSED_DGRAD_MIN_TOKENS:
            self.wt = TransposedShadows(self.param_tensors)
            self.wt.attach(self.param_tensors)
            self.wt.refresh()
        self.grad_tensors: ModelTensors = collect(views_g, c.depth, c.dim)
        if not c.learn_temb:
            self.grad_tensors.temb = None
        self._temb_t: List[torch.Tensor] = []
        # gradient arena below this element is accumulated (embeddings: atomics in the
        # embedding backward); above it every range has a single writer per step
        self.acc_hi = min(self.offsets[n][0] for n in self.names if n.rsplit(".", 1)[0] in ln_prefixes)
        # time_embed rows no sample can select (t >= temb_rows: cold diffusion draws
        # t in 1..log2 W): zero gradient and zero Adam moments for the whole run, so
        # AdamW reduces to p *= (1 - lr wd).  The optimizer skips them and
        # accumulates that factor on the device (lazy_decay); materialize_lazy()
        # applies it before anything reads them (end of train_steps, snapshots,
        # state dicts).  ~11 % of the ViT-tiny arena.
        self.lazy = None
        self.lazy_decay = torch.ones(1, dtype=torch.float32, device=self.device)
        self._lazy_dirty = False
        rows = self.cfg.temb_rows
        if (rows is not None and 0 < rows < c.total_steps and "time_embed.weight" in self.offsets
                and "time_embed.weight" not in self.frozen):
            to, tn = self.offsets["time_embed.weight"]
            lo, hi = (to + rows * c.dim + 3) // 4 * 4, (to + tn) // 4 * 4
            if hi > lo and hi <= self.train_hi:
                self.lazy = (lo, hi)
        # LayerNorm dgamma/dbeta replica workspace in backward order: final norm,
        # then norm2, norm1 of blocks L-1 .. 0; destinations = grad-arena views
        # (weight and bias of one LayerNorm are adjacent: one [2D] range).
        D = c.dim
        L = c.depth
        order = ["norm"]
        for i in range(L - 1, -1, -1):
            order += [f"blocks.{i}.norm2", f"blocks.{i}.norm1"]
        self.ln_order = order
        dsts = []
        for nm in order:
            ow, _ = self.offsets[nm + ".weight"]
            ob, _ = self.offsets[nm + ".bias"]
            assert ob == ow + D, "LayerNorm weight/bias must be adjacent in the arena"
            dsts.append(self.flat_g[ow:ow + 2 * D])
        self.ln_dsts = dsts
        # workspace rows depend on the backward's row count (ops.ln_ws_rows): allocated by
        # _ensure_ln_ws at the first step of a batch size (eager, never inside a capture)
        self.ln_ws = None
        self.ln_R = 0
        self.ln_ptrs = torch.tensor([t.data_ptr() for t in dsts], dtype=torch.int64, device=dev) \
            if dev.type == "cuda" else None
        self._ln_prefixes = ln_prefixes
        self._build_buckets()

    def _ensure_batch_buffers(self, B: int):
        """Buffers sized by the batch: the LayerNorm dgamma/dbeta slot workspaces
        ([2L+1, ops.ln_ws_rows(B N), 2D]) and room in the grad-norm partials for the
        embedding workgroups of the weight-gradient launch (FUSE_EMBED_WGRAD)."""
        c = self.prog.cfg
        D, M = c.dim, B * c.tokens
        rows = ops.ln_ws_rows(M)
        nparts = ops.sq_parts_size(self._sq_tiles + ops.wgrad_embed_slots(
            B, c.tokens, D, self._emb_owners(B), len(self.ln_order), 2 * D, M >= 16384))
        if (self.ln_ws is not None and self.ln_ws.shape[1] == rows and self.sqnorm.numel() >= nparts):
            return
        if self.is_cuda and torch.cuda.is_current_stream_capturing():
            raise RuntimeError("the batch size changed inside a graph capture (LayerNorm workspace)")
        self.ln_ws = torch.zeros(len(self.ln_order), rows, 2 * D, dtype=torch.float32, device=self.device)
        self.ln_R = rows
        if self.sqnorm.numel() < nparts:
            self.sqnorm = torch.zeros(nparts, dtype=torch.float32, device=self.device)

    def _ln_offs(self):
        """Arena offsets (elements, from the optimizer's gradient view) of the LayerNorm
        gradient ranges, in ``ln_order``."""
        base = self.opt_g.data_ptr()
        return [(d.data_ptr() - base) // 4 for d in self.ln_dsts]

    def _emb_owners(self, B: int) -> int:
        """Distinct timesteps a batch of ``B`` can hold (time-embedding gradient rows)."""
        rows = self.cfg.temb_rows
        return max(1, min(B, rows if rows is not None else self.prog.cfg.total_steps))

    def _build_buckets(self):
        """All-reduce bucket layout from ``cfg.bucket_blocks`` / ``cfg.embed_bucket``
        (re-run by :meth:`set_comm_layout`)."""
        c = self.prog.cfg
        # all-reduce buckets: contiguous arena ranges, boundaries after block groups (backward order)
        L = c.depth
        # a block's arena range starts at its first Linear weight (LayerNorms live
        # with the embeddings, see the layout above)
        starts = [min(self.offsets[n][0] for n in self.names if n.startswith(f"blocks.{i}.")
                      and n.rsplit(".", 1)[0] not in self._ln_prefixes) for i in range(L)]
        bb = max(1, self.cfg.bucket_blocks)
        self.bucket_after: Dict[int, int] = {}
        bounds = []
        end = self.train_hi  # frozen tensors (past train_hi) are never reduced
        j = 0
        for i in range(L - 1, -1, -1):
            if ((L - 1 - i) % bb == bb - 1 and i > 0) or (i == 0 and self.cfg.embed_bucket):
                bounds.append((starts[i], end))
                self.bucket_after[i] = j
                end = starts[i]
                j += 1
        bounds.append((0, end))
        self.bucket_after[-1] = j
        self.buckets = bounds
        # sub-ranges actually all-reduced per bucket (inactive time_embed rows skipped)
        self.bucket_ranges = []
        to, tn = self.offsets["time_embed.weight"]
        rows = self.cfg.temb_rows
        skip = None
        if rows is not None and 0 < rows < self.prog.cfg.total_steps:
            skip = (to + rows * c.dim, to + tn)
        for a, b in bounds:
            if skip is not None and a <= skip[0] and skip[1] <= b:
                self.bucket_ranges.append([r for r in ((a, skip[0]), (skip[1], b)) if r[1] > r[0]])
            else:
                self.bucket_ranges.append([(a, b)])
        self.temb_bucket = None
        if (self.cfg.temb_sparse and self.segmented and self.grad_tensors.temb is not None
                and (rows is None or rows >= self.prog.cfg.total_steps)):
            for k, (a, b) in enumerate(bounds):
                if a <= to and to + tn <= b:
                    self.temb_bucket = k
                    self.bucket_ranges[k] = [r for a2, b2 in self.bucket_ranges[k]
                                             for r in ((a2, min(b2, to)), (max(a2, to + tn), b2)) if r[1] > r[0]]
        # LN index range finalised at each bucket boundary (backward order)
        self.ln_done_at = {}
        done = 1
        for i in range(L - 1, -1, -1):
            done += 2
            if i in self.bucket_after:
                self.ln_done_at[i] = done
        self.ln_done_at[-1] = len(self.ln_order)

    def _refresh_shadow(self):
        self.flat_pb.copy_(self.flat_p.to(torch.bfloat16))
        if getattr(self, "lnfold", None) is not None:
            self.lnfold.refresh()
        if getattr(self, "wt", None) is not None:
            self.wt.refresh()

    # ------------------------------------------------------------------ step program
    def set_batch_fn(self, fn: Callable):
        """``fn() -> (x_t, target, t)`` device tensors; called inside the captured region."""
        self.batch_fn = fn
        self._graphs = None
        self._multi = None

    def _grad_overwrite(self, k_acc: int, deferred: bool, ln_final) -> bool:
        """One micro-batch, deferred weight gradients (the single-process tail launch or
        one launch per data-parallel bucket) and the LayerNorm finalize in the
        embedding launch: everything above ``acc_hi`` in the gradient arena
        (LayerNorms, blocks, head) is written by exactly one producer per step, which
        then stores instead of adding -- the optimizer zeroes only the embeddings
        (accumulated by atomics) and the deferred launches read no gradients.  The
        all-reduce sums the fresh values in place."""
        return self.is_cuda and k_acc == 1 and deferred and ln_final is not None

    def _step_iter(self):
        c = self.prog.cfg
        k_acc = max(1, int(self.cfg.grad_accum))
        # loss bookkeeping + counter advance ride in the LayerNorm-fold launch after
        # the optimizer (one workgroup of it) instead of two extra tiny launches.
        # With grad_accum > 1 the micro-batch loss partials are averaged first, so the
        # EMA moves once per optimizer step (multi_gpu_trainer.py:126 semantics).
        tail = self.lnfold is not None
        loss_acc = None
        overwrite = False
        self._temb_t = []
        for micro in range(k_acc):
            last = micro == k_acc - 1
            if micro > 0:
                self.rng[1:].add_(1)  # fresh dropout masks and batch draws per micro-batch
            fused_loss = tail and self.prog.supports_fused_loss(self.param_tensors)
            spec = getattr(self.batch_fn, "fused_spec", None)
            cold = None
            if fused_loss and self.cfg.fuse_batch and spec is not None:
                (img, tgt, t), cold = spec()  # drawn inside the patch-embedding launch
            else:
                img, tgt, t = self.batch_fn()
            self._temb_t.append(t)
            self._ensure_batch_buffers(int(t.shape[0]))
            if fused_loss:
                # head GEMM epilogue computes the loss partials and the token-layout gradient
                (loss_parts, dtok), S = self.prog.forward(self.param_tensors, img, t, self.rng, True,
                                                          loss=(tgt, self.cfg.loss_beta), cold=cold)
                out = None
            else:
                out, S = self.prog.forward(self.param_tensors, img, t, self.rng, True)
            if out is None:
                pass
            elif tail or k_acc > 1:
                loss_parts, dtok = ops.smooth_l1_fwd_bwd(out, tgt, c.tokens, c.patch, self.cfg.loss_beta,
                                                         finish=False)
            else:
                _, dtok = ops.smooth_l1_fwd_bwd(out, tgt, c.tokens, c.patch, self.cfg.loss_beta, self.loss_last,
                                                self.loss_ema, self.cfg.ema_decay)
            del out
            if k_acc > 1:  # mean over micro-batches (partials sum to each micro-batch's loss)
                lp = loss_parts.float() * (1.0 / k_acc)
                loss_acc = lp if loss_acc is None else loss_acc + lp
            ln_lo = 0
            # without a separate embedding bucket (single process) the patch-embedding
            # weight gradient joins block 0's grouped launch
            merge = not (self.segmented and self.cfg.embed_bucket)
            # the LayerNorm replica finalize rides in the embedding-backward launch (data
            # parallel too: every LayerNorm lives in the last bucket's arena range)
            ln_final = None
            if self.ln_ptrs is not None and FUSE_LN_FINAL:
                hi = self.ln_done_at[-1]
                ln_final = (self.ln_ws[:hi], self.ln_ptrs[:hi], 2 * c.dim, self.ln_R)
            # single process: every weight gradient in one launch after the backward (no
            # bucket needs a block's gradients early); data parallel: one launch per
            # gradient bucket, so its all-reduce can start while the backward goes on
            flush_at = set(k for k in self.bucket_after if k >= 0) if self.segmented else None
            # one micro-batch: every gradient above the embeddings has ONE producer per
            # step (the deferred weight-gradient launches, the LayerNorm finalize), so those
            # write instead of accumulate and the optimizer zeroes only the embeddings
            overwrite = self._grad_overwrite(k_acc, True, ln_final)
            if overwrite:
                ln_final = ln_final + (True,)
            # single process, one micro-batch: the deferred weight-gradient launch is the
            # last writer of the gradient arena and writes the grad-norm partials too
            fuse_sq = (FUSE_SQNORM and overwrite and flush_at is None and k_acc == 1 and self.world == 1
                       and self.is_cuda)
            B = int(t.shape[0])
            emb_fused = None
            if (fuse_sq and FUSE_EMBED_WGRAD and merge and self.grad_tensors.temb is not None and B <= 256
                    and ln_final is not None):
                emb_fused = (self._emb_owners(B), self._ln_offs()[:ln_final[1].numel()])
            for i in self.prog.backward_iter(self.param_tensors, self.grad_tensors, S, dtok, self.rng, True,
                                             ln_ws=self.ln_ws, embed_with_block0=merge, ln_final=ln_final,
                                             wgrad_flush=flush_at, wgrad_store=overwrite,
                                             wgrad_sq=(self.sqnorm, self.opt_g, self.lazy) if fuse_sq else None,
                                             embed_fused=emb_fused):
                if i in self.bucket_after and (self.segmented or i == -1):
                    hi = self.ln_done_at[i]
                    if ln_final is not None:
                        ln_lo = hi  # already finalized by the embedding backward
                    if hi > ln_lo:
                        ops.replica_reduce_(self.ln_ws[ln_lo:hi],
                                            None if self.ln_ptrs is None else self.ln_ptrs[ln_lo:hi],
                                            2 * c.dim, self.ln_R, dsts=self.ln_dsts[ln_lo:hi])
                        ln_lo = hi
                    if last:
                        yield ("bucket", self.bucket_after[i])
            S = None
        # optimizer: grads are SUM-reduced over ranks and summed over micro-batches
        # -> average via grad_scale
        gs = 1.0 / (self.world * k_acc)
        if not fuse_sq:
            ops.sqnorm(self.opt_g, self.sqnorm, gs, lazy=self.lazy)
        if loss_acc is not None:
            loss_parts = loss_acc
        ops.adamw_step(self.opt_p, self.opt_g, self.opt_m, self.opt_v, self.opt_pb, self.sqnorm,
                       self.step_ctr, self.hyper, gs, zero_hi=self.acc_hi if overwrite else None,
                       lazy=self.lazy, lazy_decay=self.lazy_decay)
        if self.wt is not None:  # the input-gradient GEMMs' transposed shadows of the new weights
            self.wt.refresh()
        if tail:
            self.lnfold.refresh(tail=(loss_parts, self.loss_last, self.loss_ema, self.cfg.ema_decay, self.step_ctr,
                                      self.rng, self.sqnorm))
        else:
            if k_acc > 1:  # one EMA update per optimizer step
                loss = loss_parts.sum().reshape(self.loss_last.shape)
                self.loss_last.copy_(loss)
                self.loss_ema.mul_(self.cfg.ema_decay).add_(loss, alpha=1.0 - self.cfg.ema_decay)
            if self.lnfold is not None:
                self.lnfold.refresh()
            ops.advance_counters(self.step_ctr, self.rng, self.sqnorm)
        self.prog._keep = None
        yield ("done", -1)

    def _allreduce(self, k: int, after=None):
        """Issue bucket ``k``'s collectives on the comm stream, ordered after the
        current stream (or after the event ``after``: the bucket's boundary inside
        the replayed compute graph)."""
        if self.ncomm is None and (not self.dist_on or (self.world <= 1 and not self.cfg.force_segments)):
            return
        ranges = self.bucket_ranges[k]

        fake = os.environ.get("DDIM_COLD_FAKE_COMM") == "1"

        def reduce():
            many = getattr(self.ncomm, "all_reduce_many_", None)
            if many is not None and self.flat_gw is None and not fake and len(ranges) > 1:
                # the bucket's ranges as one RCCL group: one launch
                many([self.flat_g[a:b] for a, b in ranges])
                if k == self.temb_bucket:
                    self._temb_exchange()
                return
            for a, b in ranges:
                if fake:  # topology experiment at 1 rank: passes over the range stand in for the collective
                    self.flat_g[a:b].mul_(1.0)
                elif self.ncomm is not None:
                    if self.flat_gw is None:
                        self.ncomm.all_reduce_(self.flat_g[a:b])
                    else:
                        self.ncomm.all_reduce_bf16_wire_(self.flat_g[a:b], self.flat_gw[a:b])
                elif self.flat_gw is None:
                    dist.all_reduce(self.flat_g[a:b], group=self.pg)
                else:  # bf16 wire: fused pack, reduce, fused unpack (on the comm stream)
                    w = self.flat_gw[a:b]
                    ops.wire_pack(self.flat_g[a:b], w)
                    dist.all_reduce(w, group=self.pg)
                    ops.wire_unpack(w, self.flat_g[a:b])
            if k == self.temb_bucket:
                self._temb_exchange()

        if self.comm is not None:
            if after is not None:
                after.wait(self.comm)
            else:
                self.comm.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self.comm):
                reduce()
        else:
            reduce()

    def _temb_exchange(self):
        """Sum the time_embed gradient over ranks from its non-zero rows only.

        Each rank contributes (t, row) for the distinct timesteps of its micro-batches
        (a repeated t keeps its first row, which already holds every sample's
        contribution), all-gathered; every rank then forms each gathered row's total
        with one [W*n, W*n] 0/1 matrix product over the gathered rows -- the same
        inputs and the same kernel on every rank, so the replicas stay bit-identical
        (a scatter-add with atomics would round differently per rank) -- and writes it
        back to those rows.  Rows no rank touched are zero everywhere already."""
        g = self.grad_tensors.temb
        idx = torch.cat([t.reshape(-1) for t in self._temb_t]).to(torch.int64)
        n = idx.numel()
        rows = g.index_select(0, idx)
        first = ~(idx[:, None] == idx[None, :]).tril(-1).any(1)
        rows.mul_(first[:, None].to(rows.dtype))
        idx_all = idx.new_empty(self.world * n)
        rows_all = rows.new_empty(self.world * n, g.shape[1])
        if self.ncomm is not None:  # every per-step collective on the one gradient communicator
            self.ncomm.all_gather_(idx_all, idx)
            self.ncomm.all_gather_(rows_all, rows)
        else:
            dist.all_gather_into_tensor(idx_all, idx, group=self.pg)
            dist.all_gather_into_tensor(rows_all, rows, group=self.pg)
        same = (idx_all[:, None] == idx_all[None, :]).to(rows.dtype)
        g.index_copy_(0, idx_all, same @ rows_all)

    def _join_comm(self):
        if self.comm is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.comm)

    # ------------------------------------------------------------------ comm layout
    # candidate gradient-exchange layouts for autotune_comm(): (name, bucket_blocks,
    # embed_bucket, inline).  overlap-*: buckets of 2 / 4 blocks + the embeddings,
    # all-reduced on the comm stream while the backward goes on; inline-1: ONE
    # all-reduce of the whole arena on the compute stream after the backward (no
    # second queue: the single-process step + the collective).  These run
    # event-split: collectives host-issued between the step's two graphs.
    # graph-inline-1: the same single all-reduce CAPTURED on the compute stream
    # inside the step graph -- one linear graph, no second queue, no host hand-off,
    # so ``graph_steps`` K-step graphs work data parallel too (the event-split
    # layouts replay two graphs per step).  graph-<overlap>: the captured comm-stream
    # branch (a fork/join per bucket inside the graph, K-step graphs as well).
    COMM_LAYOUTS = (("graph-inline-1", 1 << 16, False, True), ("overlap-2", 2, True, False),
                    ("overlap-4", 4, True, False), ("inline-1", 1 << 16, False, True))

    @classmethod
    def layout_by_name(cls, name: str):
        """``(name, bucket_blocks, embed_bucket, inline)`` for ``[graph-]overlap-<blocks>``
        / ``[graph-]inline-1`` (``graph-``: collectives captured in the step graph)."""
        base = name[6:] if name.startswith("graph-") else name
        if base == "inline-1":
            return (name, 1 << 16, False, True)
        if base.startswith("overlap-") and base[8:].isdigit() and int(base[8:]) >= 1:
            return (name, int(base[8:]), True, False)
        raise ValueError(f"unknown gradient-exchange layout {name!r} ([graph-]overlap-<blocks> or "
                         "[graph-]inline-1)")

    def _comm_capturable(self) -> bool:
        """Can the gradient collectives be captured into a hipGraph?  RCCL (our
        communicator or ProcessGroupNCCL) and the device loopback pair can; gloo
        stages CUDA tensors through the host and aborts the process inside a capture."""
        if self.ncomm is not None:
            return True
        try:
            return self.dist_on and dist.get_backend(self.pg) == "nccl"
        except Exception:  # pragma: no cover
            return False

    def apply_layout(self, layout):
        """Switch to a layout given by name or ``(name, bucket_blocks, embed_bucket,
        inline[, ...])``; records it as :attr:`comm_choice`.  A captured (``graph-``)
        layout on a non-capturable backend (gloo) runs as its event-split form."""
        L = self.layout_by_name(layout) if isinstance(layout, str) else tuple(layout)
        captured = L[0].startswith("graph-")
        if captured and self.is_cuda and self.segmented and not self._comm_capturable():
            import warnings
            warnings.warn(f"layout {L[0]}: collectives of this backend cannot be captured in a hipGraph; "
                          f"running {L[0][6:]} (event-split)")
            L = (L[0][6:],) + tuple(L[1:])
            captured = False
        self.set_comm_layout(L[1], L[2], L[3], captured=captured)
        self.comm_choice = L[0]
        return L

    def step_profile(self):
        """Cost-model view of this engine's step (parallel.costmodel.StepProfile):
        gradient bytes per block and of the rest (embeddings, head, LayerNorms,
        active time_embed rows) on the wire, backward timing scaled from the
        measured ViT-tiny step by this batch's GEMM work."""
        from ..parallel import costmodel as cm
        c = self.prog.cfg
        wire = 2 if self.cfg.grad_wire == "bf16" else 4
        hidden = self.offsets["blocks.0.mlp.fc1.bias"][1]
        xb = getattr(self.batch_fn, "x_t", None)
        B = int(xb.shape[0]) if isinstance(xb, torch.Tensor) else 32
        prof = cm.vit_step_profile(c.depth, c.dim, hidden, B * c.tokens, 0, wire_bytes=wire)
        head = sum(self.offsets[n][1] for n in ("head.weight", "head.bias") if n in self.offsets)
        prof.head_bytes = float(head * wire)
        other = max(0.0, self.reduced_numel() - c.depth * prof.block_bytes / wire - head)
        prof.embed_bytes = float(other * wire)
        return prof

    def reduced_numel(self) -> int:
        """Elements all-reduced per step (inactive time_embed rows / frozen tensors skipped)."""
        return sum(b - a for rs in self.bucket_ranges for a, b in rs)

    def probe_allreduce(self, sizes_mb=(0.25, 1.0, 4.0, 16.0), reps: int = 10):
        """Measure the gradient all-reduce on THIS job's ranks (the engine's own comm
        path: native RCCL communicator or torch.distributed, fp32) at a few sizes and
        fit ``T = alpha + S / algbw`` (parallel.costmodel.fit_allreduce).  Max over
        ranks, HIP-event timed on the stream the collectives run on (host clock for
        gloo on the CPU).  Returns the fitted model and ``{bytes: us}``; ``(None, {})``
        when not data parallel."""
        if not (self.dist_on and self.world > 1):
            return None, {}
        import time
        from ..parallel import costmodel as cm
        from ..parallel.dist import all_reduce_max, barrier
        n_max = int(max(sizes_mb) * (1 << 20) // 4)
        buf = torch.zeros(n_max, dtype=torch.float32, device=self.device)
        out = {}

        def sync():
            if self.is_cuda:
                torch.cuda.synchronize(self.device)
        for mb in sizes_mb:
            n = int(mb * (1 << 20) // 4)
            x = buf[:n]

            def ar():
                if self.ncomm is not None:
                    self.ncomm.all_reduce_(x)
                else:
                    dist.all_reduce(x, group=self.pg)
            for _ in range(3):
                ar()
            sync()
            barrier()
            if self.is_cuda:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    ar()
                e1.record()
                sync()
                us = e0.elapsed_time(e1) * 1e3 / reps
            else:  # gloo on the CPU: host clock
                t0 = time.perf_counter()
                for _ in range(reps):
                    ar()
                us = (time.perf_counter() - t0) * 1e6 / reps
            out[4 * n] = all_reduce_max(us, self.device)
        del buf
        fit = cm.fit_allreduce(self.world, list(out), list(out.values()))
        self.comm_fit = fit
        return fit, out

    def model_layouts(self, model=None):
        """Layouts ordered by the cost model's predicted exposed comm time:
        ``[(name, bucket_blocks, embed_bucket, inline, exposed_us)]``; ``model`` =
        the fitted all-reduce model (:meth:`probe_allreduce`) or the a-priori xGMI
        ring model of this world size."""
        from ..parallel import costmodel as cm
        if model is None:
            model = getattr(self, "comm_fit", None) or cm.xgmi_ring_model(max(2, min(self.world, 8)))
        return cm.plan_buckets(self.step_profile(), model)

    def candidate_layouts(self):
        """autotune_comm()'s default candidates: :attr:`COMM_LAYOUTS` plus the cost
        model's predicted best (fitted model if :meth:`probe_allreduce` ran)."""
        cands = list(self.COMM_LAYOUTS)
        if self.is_cuda and self.segmented and not self._comm_capturable():
            cands = [L_ for L_ in cands if not L_[0].startswith("graph-")]
        best = self.model_layouts()[0]
        if best[0] not in [L_[0] for L_ in cands]:
            cands.insert(1, best[:4])  # right after graph-inline-1 (the time budget runs in order)
        return cands

    def set_comm_layout(self, bucket_blocks: Optional[int] = None, embed_bucket: Optional[bool] = None,
                        inline: Optional[bool] = None, captured: Optional[bool] = None):
        """Re-bucket the gradient all-reduce and choose where its collectives run (a
        comm-stream branch overlapping the backward, or inline on the compute
        stream) and how (``captured``: inside the step graph; else host-issued
        between the event-split graphs).  The step graphs are dropped and
        re-captured after ``graph_warmup`` eager steps of the new layout."""
        import dataclasses
        kw = {}
        if bucket_blocks is not None:
            kw["bucket_blocks"] = int(bucket_blocks)
        if embed_bucket is not None:
            kw["embed_bucket"] = bool(embed_bucket)
        if inline is not None:
            kw["comm_inline"] = bool(inline)
        if captured is not None:
            kw["comm_events"] = not captured
            kw["graph_comm"] = bool(captured)
        if self.is_cuda:
            torch.cuda.synchronize(self.device)
        self.cfg = dataclasses.replace(self.cfg, **kw)
        self._build_buckets()
        if self.is_cuda and self.segmented:
            self.comm = None if self.cfg.comm_inline else self._comm_obj
        self._graphs = None
        self._multi = None
        self._events = None
        self._signal = None
        self._eager_steps = 0
        self._graph_comm_failed = False

    def _snapshot_state(self):
        self.materialize_lazy()
        keys = ("flat_p", "flat_g", "flat_m", "flat_v", "rng", "step_ctr", "loss_ema", "loss_last", "lazy_decay")
        return {k: getattr(self, k).clone() for k in keys}, self.steps_done

    def _restore_state(self, snap):
        tensors, steps = snap
        for k, v in tensors.items():
            getattr(self, k).copy_(v)
        self.steps_done = steps
        self._lazy_dirty = False  # snapshots are taken materialized
        self._refresh_shadow()

    def autotune_comm(self, steps: int = 100, warm: int = 10, layouts=None, budget_s: Optional[float] = None):
        """Pick the gradient-exchange layout by measuring it on THIS job's ranks.

        Every layout of ``layouts`` (default :meth:`candidate_layouts`) runs
        ``graph_warmup`` eager steps, its capture and ``warm`` replayed steps, is
        checked, then timed over ``steps`` optimizer steps; the time is the max over
        ranks (so every rank takes the same decision) and the fastest layout is kept.
        Fail-fast, so the tuning can never eat the job's time limit:

        * a layout whose warm-up raised (a capture the RCCL build refuses) or whose
          counter hand-off timed out on ANY rank is dropped right after the warm-up
          (the timed-out wait raises the error word; every later wait then returns
          at once, so a broken layout costs one timeout, not one per bucket and step);
        * ``budget_s`` (default ``DDIM_COLD_AUTOTUNE_BUDGET_S``, 30 s) bounds the whole
          tuning: once spent (max over ranks), the remaining candidates are skipped;
        * if NO layout ran, the engine does not raise: it falls back to
          :meth:`fallback_eager_inline` (no graphs, no hand-offs, one all-reduce on the
          compute stream; on torch.distributed's communicator if ours fails too) and
          records the reason in :attr:`comm_fallback`.

        Parameters, Adam moments, counters, RNG and loss EMA are restored afterwards:
        the tuning steps leave no trace in the training state.  Returns
        ``{name: ms_per_step}`` (``inf``: failed, ``nan``: skipped for time; empty
        when not data parallel on a GPU).  Testing: ``DDIM_COLD_TEST_FAIL_LAYOUTS=1``
        makes every candidate fail after its warm-up."""
        if not (self.segmented and self.is_cuda and self.dist_on):
            return {}
        import time
        import warnings
        from ..parallel.dist import all_reduce_max, barrier
        from ..parallel.watchdog import phase
        if budget_s is None:
            budget_s = float(os.environ.get("DDIM_COLD_AUTOTUNE_BUDGET_S", "30"))
        force_fail = os.environ.get("DDIM_COLD_TEST_FAIL_LAYOUTS") == "1"
        layouts = list(layouts or self.candidate_layouts())
        snap = self._snapshot_state()
        times: Dict[str, float] = {}
        self.autotune_errors: Dict[str, str] = {}
        t_begin = time.perf_counter()
        for L in layouts:
            name = L[0]
            if all_reduce_max(time.perf_counter() - t_begin, self.device) > budget_s:
                times[name] = math.nan
                continue
            phase(f"autotune:{name}")
            failed = 0.0
            try:
                self.apply_layout(L)
                self.train_steps(self.cfg.graph_warmup + warm)
                if force_fail:
                    raise RuntimeError("DDIM_COLD_TEST_FAIL_LAYOUTS=1 (test hook)")
                torch.cuda.synchronize(self.device)
                if self.comm_error():
                    failed = 1.0
                    self.autotune_errors[name] = "hand-off wait timed out"
            except Exception as e:  # noqa: BLE001 - a candidate that cannot run is dropped, not fatal
                failed = 1.0
                self.autotune_errors[name] = repr(e)[:300]
                torch.cuda.synchronize(self.device)
            # every rank drops the layout if it failed on ANY rank; its stale-gradient
            # steps are undone by the state restore below
            if all_reduce_max(failed, self.device) > 0:
                times[name] = math.inf
                self.reset_comm_error()
                continue
            barrier()
            t0 = time.perf_counter()
            self.train_steps(steps)
            torch.cuda.synchronize(self.device)
            dt = time.perf_counter() - t0
            if self.comm_error():
                dt = math.inf
            times[name] = all_reduce_max(dt, self.device) / steps * 1e3
            self.reset_comm_error()
        ok = [L_ for L_ in layouts if math.isfinite(times[L_[0]])]
        self._restore_state(snap)
        for name, err in self.autotune_errors.items():
            warnings.warn(f"autotune_comm: layout {name} dropped ({err})")
        self.comm_times = times
        if not ok:
            warnings.warn(f"autotune_comm: no gradient-exchange layout ran ({times}); falling back to the "
                          "eager inline all-reduce")
            self.fallback_eager_inline(f"no layout ran: {sorted(self.autotune_errors)}")
        else:
            best = min(ok, key=lambda L_: times[L_[0]])
            self.apply_layout(best)
            phase("autotune:chosen", layout=best[0], ms=round(times[best[0]], 4))
        self.autotune_s = time.perf_counter() - t_begin
        return times

    def fallback_eager_inline(self, reason: str, verify_steps: int = 2):
        """Last-resort data-parallel step: no hipGraphs, no comm stream, no counter
        hand-offs -- forward + backward eagerly, then ONE all-reduce of the whole
        gradient arena on the compute stream, then the optimizer (the reference's
        DDP step minus the bucket overlap).  ``verify_steps`` eager steps are run on
        every rank (state restored afterwards); if they fail on any rank while our
        own RCCL communicator is in use, it is dropped for torch.distributed's and
        the check repeats.  Sets :attr:`comm_choice` = ``"eager-inline"`` and
        :attr:`comm_fallback` = ``reason``."""
        import dataclasses
        import warnings
        from ..parallel.dist import all_reduce_max
        from ..parallel.watchdog import phase
        phase("comm-fallback:eager-inline", reason=reason)
        self.set_comm_layout(1 << 16, False, True, captured=False)
        self.cfg = dataclasses.replace(self.cfg, use_graph=False)
        self.comm_choice = "eager-inline"
        self.comm_fallback = reason
        for attempt in range(2):
            snap = self._snapshot_state()
            failed, err = 0.0, None
            try:
                self.train_steps(verify_steps)
                if self.is_cuda:
                    torch.cuda.synchronize(self.device)
                if not bool(torch.isfinite(self.loss_last).all()):
                    failed, err = 1.0, "non-finite loss"
            except Exception as e:  # noqa: BLE001
                failed, err = 1.0, repr(e)[:300]
                if self.is_cuda:
                    torch.cuda.synchronize(self.device)
            self._restore_state(snap)
            if all_reduce_max(failed, self.device) == 0:
                phase("comm-fallback:verified", comm=self.comm_backend)
                return
            if attempt == 0 and self.ncomm is not None and self.dist_on:
                warnings.warn(f"eager inline fallback failed on the native communicator ({err}); "
                              "switching to torch.distributed")
                self.ncomm.destroy()
                self.ncomm = None
                self.comm_backend = "torch"
                self.comm_fallback = reason + "; native communicator dropped"
                continue
            break
        raise RuntimeError(f"data parallel: even the eager inline all-reduce step failed ({err}); {reason}")

    def _run_eager(self):
        gen = self._step_iter()
        for kind, k in gen:
            if kind == "bucket":
                self._allreduce(k)
                if k == len(self.buckets) - 1:
                    self._join_comm()

    def _capture(self):
        if self.segmented and self.cfg.comm_events:
            self._capture_impl(graph_comm=False, events=True)
            return
        if self.segmented and self.cfg.graph_comm and not self._graph_comm_failed:
            try:
                self._capture_impl(graph_comm=True)
                return
            except Exception as e:  # pragma: no cover - depends on the RCCL build
                if (self.comm_choice or "").startswith("graph-"):
                    # a captured layout was asked for (autotune candidate or explicit): its
                    # failure must reach autotune_comm / the caller, not be timed as segments
                    raise
                import warnings
                warnings.warn(f"capturing collectives in the step graph failed ({e!r}); "
                              "falling back to per-bucket graph segments")
                self._graph_comm_failed = True
                torch.cuda.synchronize(self.device)
        self._capture_impl(graph_comm=False)

    def _captured_step_body(self):
        """One whole step issued on the capturing stream (collectives as graph nodes)."""
        for kind, k in self._step_iter():
            if kind == "bucket":
                self._allreduce(k)
                if k == len(self.buckets) - 1:
                    self._join_comm()

    def _capture_impl(self, graph_comm: bool, events: bool = False):
        from ..utils.observe import drain_before_capture, no_gc
        if self.dist_on and self.is_cuda:
            # the warm-up's eager collectives finished on every rank (and dropped by
            # the process-group watchdog) before the capture opens
            drain_before_capture(self.device)
        with no_gc():
            if events:
                self._capture_event_graphs()
            else:
                self._capture_graphs(graph_comm)

    def _capture_event_graphs(self):
        """Compute graph (forward + backward, an external event recorded at every
        bucket boundary) + optimizer graph; see ``EngineConfig.comm_events``."""
        pool = torch.cuda.graph_pool_handle()
        nb = len(self.buckets)
        self._multi = None
        from ..parallel.comm import ExternalEvent, FlagSignal
        sig = None
        # the compute graph tells the comm stream a bucket is final by bumping a
        # per-bucket counter (a 1-lane kernel node, system-scope release) that a
        # bounded polling kernel on the comm stream waits for.  (External event-record
        # nodes were measured too: the comm stream then started only after the whole
        # compute graph, so the overlapped layouts overlapped nothing.)  Inline layout
        # (no comm stream): events only mark the bucket boundaries.
        if self.comm is not None:
            sig = FlagSignal(nb, self.device)
            evs = [sig.waiter(k) for k in range(nb)]
        else:
            evs = [ExternalEvent() for _ in range(nb)]
        gen = self._step_iter()
        g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(g1, pool=pool, capture_error_mode=CAPTURE_MODE):
            for _ in range(nb):
                kind, k = next(gen)
                assert kind == "bucket", kind
                if sig is not None:
                    sig.bump(k)
                else:
                    evs[k].record()
        with torch.cuda.graph(g2, pool=pool, capture_error_mode=CAPTURE_MODE):
            kind, _ = next(gen)
            assert kind == "done", kind
        self._graphs = [g1, g2]
        self._events = evs
        self._signal = sig
        if sig is not None:
            self.handoff_order = "pre-issued" if self._preissue_ok() else "post-replay"
        else:
            self.handoff_order = "events" if self.comm is not None else "inline"

    def _capture_graphs(self, graph_comm: bool):
        pool = torch.cuda.graph_pool_handle()
        graphs = []
        self._multi = None
        self._events = None
        self._signal = None
        gen = self._step_iter()
        nseg = len(self.buckets) + 1 if (self.segmented and not graph_comm) else 1
        if nseg == 1:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool, capture_error_mode=CAPTURE_MODE):
                self._captured_step_body()
            graphs.append(g)
            K = max(1, int(self.cfg.graph_steps))
            if K > 1:  # K steps in one graph, own memory pool
                gm = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gm, pool=torch.cuda.graph_pool_handle(), capture_error_mode=CAPTURE_MODE):
                    for _ in range(K):
                        self._captured_step_body()
                self._multi = (gm, K)
        else:
            for _ in range(nseg):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=pool, capture_error_mode=CAPTURE_MODE):
                    next(gen)
                graphs.append(g)
        self._graphs = graphs

    def _replay(self):
        gs = self._graphs
        if len(gs) == 1:
            gs[0].replay()
            return
        evs = getattr(self, "_events", None)
        if evs is not None and len(gs) == 2:
            sig = getattr(self, "_signal", None)
            if sig is not None and self.handoff_order == "pre-issued":
                # counters: the comm stream's waits + collectives can be queued BEFORE the
                # compute graph (each waits for its own counter), so the comm queue holds
                # them when the graph starts instead of receiving them behind it
                sig.expected += 1  # this replay's counter value
                for k, ev in enumerate(evs):
                    self._allreduce(k, after=ev)
                gs[0].replay()
            else:
                gs[0].replay()
                if sig is not None:
                    sig.expected += 1
                for k, ev in enumerate(evs):  # comm stream: waits on the bucket's event; inline: after gs[0]
                    self._allreduce(k, after=ev)
            self._join_comm()
            gs[1].replay()
            return
        nb = len(self.buckets)
        for k in range(nb):
            gs[k].replay()
            self._allreduce(k)
        self._join_comm()
        gs[nb].replay()

    def train_steps(self, n: int, materialize: bool = True):
        """Run ``n`` optimizer steps (``batch_fn`` draws each step's batch on the device).
        With ``graph_steps = K > 1`` every run of K steps is ONE replay of a K-step
        graph; the remainder (and the eager warm-up) goes through :meth:`train_step`.
        ``materialize``: apply the lazily accumulated weight decay afterwards (see
        ``lazy``), so every parameter is current when the call returns.
        Returns the device loss tensor of the last step (no host sync)."""
        done = 0
        while done < n:
            multi = getattr(self, "_multi", None)
            if multi is not None and n - done >= multi[1]:
                multi[0].replay()
                self.steps_done += multi[1]
                self._lazy_dirty = True
                done += multi[1]
            else:
                self.train_step(materialize=False)
                done += 1
        if materialize:
            self.materialize_lazy()
        return self.loss_last

    def materialize_lazy(self):
        """Apply the weight decay accumulated for the ``lazy`` rows since the last call
        (p *= prod(1 - lr_s wd); their moments are zero) and refresh their bf16 shadow."""
        if self.lazy is None or not self._lazy_dirty:
            return
        lo, hi = self.lazy
        self.flat_p[lo:hi].mul_(self.lazy_decay)
        self.flat_pb[lo:hi].copy_(self.flat_p[lo:hi])
        self.lazy_decay.fill_(1.0)
        self._lazy_dirty = False

    def train_step(self, materialize: bool = True):
        """Run one optimizer step on the batch produced by ``batch_fn``
        (``materialize``: as in :meth:`train_steps`; the trainer defers it to the
        epoch end, where it evaluates and checkpoints).

        Returns the device loss tensor (no host sync)."""
        if self.batch_fn is None:
            raise RuntimeError("set_batch_fn() or use step(x, target, t)")
        use_graph = self.cfg.use_graph and self.is_cuda
        if use_graph and self._graphs is None and self._eager_steps >= self.cfg.graph_warmup:
            self._capture()
        if use_graph and self._graphs is not None:
            self._replay()
        else:
            self._run_eager()
            self._eager_steps += 1
        self.steps_done += 1
        self._lazy_dirty = True
        if materialize:
            self.materialize_lazy()
        return self.loss_last

    def step(self, x_t: torch.Tensor, target: torch.Tensor, t: torch.Tensor):
        """Convenience: copy an externally produced batch into static buffers and step."""
        if self._static is None or self._static[0].shape != x_t.shape:
            self._static = (torch.empty_like(x_t, device=self.device), torch.empty_like(target, device=self.device),
                            torch.empty(t.shape, dtype=torch.int64, device=self.device))
            st = self._static
            self.set_batch_fn(lambda: st)
        sx, sy, st_ = self._static
        sx.copy_(x_t, non_blocking=True)
        sy.copy_(target, non_blocking=True)
        st_.copy_(t, non_blocking=True)
        return self.train_step()

    # ------------------------------------------------------------------ state
    def current_lr(self) -> float:
        return self._lr_at(int(self.step_ctr[1].item()))

    def _param_list(self):
        return [p for _, p in self.model.named_parameters()]

    def optimizer_state_dict(self) -> dict:
        """torch.optim.AdamW-format state dict (interchangeable with the reference's lastepoch.pkl)."""
        self.materialize_lazy()
        ctr = self.step_ctr.detach().cpu()
        return self._optimizer_sd(self.flat_m, self.flat_v, int(ctr[0]), int(ctr[1]))

    def _lr_at(self, sched_step: int) -> float:
        c = self.cfg
        if c.t_max <= 0:
            return c.lr
        return c.eta_min + (c.lr - c.eta_min) * 0.5 * (1 + math.cos(math.pi * sched_step / c.t_max))

    def _optimizer_sd(self, flat_m: torch.Tensor, flat_v: torch.Tensor, adam_step: int, sched_step: int) -> dict:
        """AdamW state dict from moment arenas (the live device ones, or a host snapshot)."""
        params = self._param_list()
        opt = torch.optim.AdamW(params, lr=self._lr_at(sched_step), betas=self.cfg.betas, eps=self.cfg.eps,
                                weight_decay=self.cfg.weight_decay)
        if adam_step > 0:
            for n, p in zip(self.names, params):
                if n in self.frozen:  # torch.optim keeps no state for a parameter without .grad
                    continue
                o, k = self.offsets[n]
                opt.state[p] = {"step": torch.tensor(float(adam_step)),
                                "exp_avg": flat_m[o:o + k].view(p.shape).clone(),
                                "exp_avg_sq": flat_v[o:o + k].view(p.shape).clone()}
        sd = opt.state_dict()
        sd["param_groups"][0]["initial_lr"] = self.cfg.lr
        return sd

    def snapshot_to_host(self) -> "HostSnapshot":
        """Training state (parameters, Adam moments, counters) for an off-critical-path
        checkpoint write: device-to-device copies into snapshot buffers on the CURRENT
        stream (ordered after the last step, ~90 MB at HBM speed for ViT-tiny), then
        device-to-host copies into pinned buffers on a side stream that the training
        stream never waits for.  ``HostSnapshot.wait()`` (the writer thread) blocks
        until the host copy has landed.  The buffers are reused: finish (wait) one
        snapshot before taking the next."""
        self.materialize_lazy()
        cur = torch.cuda.current_stream(self.device) if self.is_cuda else None
        if getattr(self, "_snap", None) is None:
            pin = self.is_cuda
            host = [torch.empty(t.shape, dtype=t.dtype, pin_memory=pin)
                    for t in (self.flat_p, self.flat_m, self.flat_v, self.step_ctr, self.rng)]
            dev = [torch.empty_like(t) for t in (self.flat_p, self.flat_m, self.flat_v, self.step_ctr, self.rng)] \
                if self.is_cuda else None
            side = torch.cuda.Stream(self.device) if self.is_cuda else None
            self._snap = (host, dev, side)
        host, dev, side = self._snap
        src = (self.flat_p, self.flat_m, self.flat_v, self.step_ctr, self.rng)
        ev = None
        if self.is_cuda:
            for d, t in zip(dev, src):
                d.copy_(t)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                for h, d in zip(host, dev):
                    h.copy_(d, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(side)
        else:
            for h, t in zip(host, src):
                h.copy_(t)
        return HostSnapshot(self, *host, ev, int(self.steps_done))

    def load_optimizer_state_dict(self, sd: dict):
        st = sd.get("state", {})
        params = self._param_list()
        step = 0
        for i, (n, p) in enumerate(zip(self.names, params)):
            s = st.get(i)
            if s is None or n in self.frozen:
                continue
            o, k = self.offsets[n]
            self.flat_m[o:o + k].copy_(s["exp_avg"].reshape(-1).to(self.device))
            self.flat_v[o:o + k].copy_(s["exp_avg_sq"].reshape(-1).to(self.device))
            step = int(float(s["step"]))
        self.step_ctr[0] = step
        self._check_lazy_moments()

    def _check_lazy_moments(self):
        """The lazy time_embed rows assume zero Adam moments for the whole run.  A
        resumed state whose moments are non-zero there (a Gaussian-diffusion run, a
        different image size / ``temb_rows``) turns the shortcut off, so those rows
        keep moving as torch.optim.AdamW would move them."""
        if self.lazy is None:
            return
        lo, hi = self.lazy
        if bool(self.flat_m[lo:hi].any()) or bool(self.flat_v[lo:hi].any()):
            import warnings
            warnings.warn("optimizer state has non-zero Adam moments on time_embed rows this run cannot "
                          "select; updating them every step (lazy weight decay off)")
            self.materialize_lazy()
            self.lazy = None
            self._graphs = None
            self._multi = None
            self._eager_steps = 0

    def scheduler_state_dict(self, sched_step: Optional[int] = None) -> dict:
        """torch CosineAnnealingLR-format state dict (at ``sched_step``, default: now).
        The key layout comes from a real scheduler built once and cached (building a
        torch optimizer costs ~1.5 s the first time in a process -- it imports the
        compiler stack -- which must not land in a background checkpoint write)."""
        if getattr(self, "_sched_template", None) is None:
            opt = torch.optim.AdamW([torch.zeros(1, requires_grad=True)], lr=self.cfg.lr)
            sch = torch.optim.lr_scheduler.CosineAnnealingLR(opt, max(self.cfg.t_max, 1), self.cfg.eta_min)
            self._sched_template = sch.state_dict()
        sd = copy.deepcopy(self._sched_template)
        sd["base_lrs"] = [self.cfg.lr]
        last = int(self.step_ctr[1].item()) if sched_step is None else int(sched_step)
        sd["last_epoch"] = last
        sd["_step_count"] = last + 1
        sd["_last_lr"] = [self._lr_at(last)]
        return sd

    def load_scheduler_state_dict(self, sd: dict):
        self.step_ctr[1] = int(sd.get("last_epoch", 0))

    def sync_params_from_model(self):
        """Call after loading weights into ``model`` (its params are arena views)."""
        self.lazy_decay.fill_(1.0)  # the loaded values are current: no decay pending
        self._lazy_dirty = False
        self._refresh_shadow()

    def detach(self):
        """Release the model from the engine (params stay on the device, as plain tensors)."""
        self.materialize_lazy()
        for n, p in self.model.named_parameters():
            p.data = p.data.clone()
            p.grad = None
        self.model._engine = None


class HostSnapshot:
    """Host copy of an engine's training state (:meth:`TrainEngine.snapshot_to_host`):
    fp32 parameter / moment arenas, counters and RNG state, plus what is needed to
    lay them out as the reference's checkpoint dicts without touching the device."""

    def __init__(self, engine: TrainEngine, p, m, v, step_ctr, rng, event, steps_done: int):
        self.engine, self.p, self.m, self.v, self.step_ctr, self.rng = engine, p, m, v, step_ctr, rng
        self.event = event
        self.steps_done = steps_done

    def wait(self):
        if self.event is not None:
            self.event.synchronize()

    def state_dict(self) -> Dict[str, torch.Tensor]:
        """The model's ``state_dict`` (parameter order and shapes) from the snapshot."""
        eng = self.engine
        shapes = {n: p.shape for n, p in eng.model.named_parameters()}
        out = {}
        for n in eng.model.state_dict().keys():
            if n not in eng.offsets:
                raise KeyError(f"{n}: not in the parameter arena (a buffer?) -- snapshot cannot hold it")
            o, k = eng.offsets[n]
            out[n] = self.p[o:o + k].view(shapes[n]).clone()
        return out

    def optimizer_state_dict(self) -> dict:
        return self.engine._optimizer_sd(self.m, self.v, int(self.step_ctr[0]), int(self.step_ctr[1]))

    def scheduler_state_dict(self) -> dict:
        return self.engine.scheduler_state_dict(int(self.step_ctr[1]))
