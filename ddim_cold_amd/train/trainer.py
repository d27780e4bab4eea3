"""Experiment trainer: the reference's ``multi_gpu_trainer.main`` semantics on the MI355X engine.

Reference flow (multi_gpu_trainer.py:47-165) reproduced:

* process group per rank (RCCL on GPUs, gloo on CPU), shared init weights file
  (rank 0 writes ``<SavedDir>/<initializing>`` if absent; here a barrier instead
  of ``sleep(5)``, and a load failure is an error instead of a swallowed print),
* log header (``Date``, ``TrainSet batchs``, ``TestSet batchs``),
* AdamW(wd 0.05) + cosine LR over ``steps_per_epoch * epoch_end`` stepped per
  iteration + clip 1.0, smooth-L1 loss, loss EMA ``0.99/0.01`` from 5.0,
* every ``log_every`` (100) steps: ``steps: .. loss: .. time_cost: ..`` (rank 0),
* per epoch: eval mean smooth-L1 over the val shard, SUM-all-reduced / world,
  ``epoch: .. loss: ..``, scalar ``loss``, ``bestloss.pkl`` on improvement and
  ``lastepoch.pkl`` every epoch (rank 0),
* resume from ``resume:`` (epoch+1, loss_rec, steps, best metric, optimizer,
  scheduler).

MI355X differences: batches are formed on the device from a decoded image
cache (or a synthetic pool) with DistributedSampler index semantics, the step
runs as replayed hipGraphs, and the loss is read back only at log points
(no per-step ``print(loss)`` / ``.item()`` sync).
"""
from __future__ import annotations

import math
import os
import shutil
import time
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

from .. import ops
from ..config import ExperimentConfig
from ..data.datasets import DeviceImageCache, shard_indices
from ..data.synthetic import SITE_DATA, make_batcher, synthetic_pool
from ..models.program import model_tensors
from ..models.vit import DiffusionVisionTransformer
from ..parallel import dist as pdist
from ..utils.logging import ScalarWriter, asctime, fmt_epoch, fmt_steps, printLog
from ..utils.observe import FaultInjected, StepClock, check_param_sync, phase, torch_profiler
from . import checkpoint as ckpt
from .engine import CAPTURE_MODE, EngineConfig, TrainEngine


@dataclass
class Paths:
    saved_dir: str       # reference SavedDir (``Saved_Models/``)
    ckpt_dir: str        # reference CheckpointDir (``Saved_Models/<Exp><framework>/``)
    log: str             # train.log

    @classmethod
    def make(cls, cfg: ExperimentConfig, exp_name: str, root: Optional[str] = None, config_path: Optional[str] = None):
        saved = cfg.ckpt_dir or os.path.join(root or os.getcwd(), "Saved_Models")
        saved = saved.rstrip("/") + "/"
        cdir = os.path.join(saved, exp_name + cfg.framework) + "/"
        os.makedirs(cdir, exist_ok=True)
        if config_path and os.path.isfile(config_path):
            try:
                shutil.copy(config_path, cdir)
            except shutil.SameFileError:
                pass
        return cls(saved, cdir, os.path.join(cdir, "train.log"))


def _device_for(rank: int, local_rank: int, backend: Optional[str]) -> torch.device:
    if backend == "gloo" or not torch.cuda.is_available():
        return torch.device("cpu")
    return torch.device("cuda", local_rank)


def _pools(cfg: ExperimentConfig, device, rank: int):
    size = tuple(cfg.image_size)
    if cfg.synthetic:
        train = synthetic_pool(cfg.synthetic_size, size, seed=cfg.seed, device=device)
        val = synthetic_pool(max(cfg.synthetic_size // 8, 1), size, seed=cfg.seed + 1, device=device)
        return train, val
    tr = DeviceImageCache(cfg.dataStorage[0], size, device, workers=cfg.num_workers)
    va = DeviceImageCache(cfg.dataStorage[1], size, device, workers=cfg.num_workers)
    return tr.float_pool(), va.float_pool()


EVAL_GROUP = 8  # validation batches per captured evaluation replay (see evaluate)


def _eval_batch(prog, P, src, eval_rng, total):
    """One validation batch: draw, eval-mode forward, smooth-L1 added to ``total`` (device)."""
    c = prog.cfg
    x_t, target, t = src()
    out, _ = prog.forward(P, x_t, t, eval_rng, False, save=False)
    if out.is_cuda:
        loss, _ = ops.smooth_l1_fwd_bwd(out, target, c.tokens, c.patch, 1.0)
    else:
        loss = torch.nn.functional.smooth_l1_loss(out, target).reshape(1)
    total += loss.double()
    eval_rng[1:].add_(1)


@torch.no_grad()
def evaluate(model, engine: TrainEngine, pool: torch.Tensor, idx: torch.Tensor, batch: int, kind: str,
             total_steps: int, eval_rng: torch.Tensor) -> float:
    """Mean per-batch smooth-L1 over ``pool[idx]`` in eval mode (multi_gpu_trainer.py:32-45).

    On a GPU every EVAL_GROUP full batches are one replay of a captured graph (batch
    draw from a static index buffer, one forward, loss accumulated on the device;
    captured once per (pool, batch, kind) and kept on the engine); the remaining
    batches run eagerly.  One host sync at the end."""
    prog = engine.prog
    P = engine.param_tensors
    dev = pool.device
    total = torch.zeros(1, dtype=torch.float64, device=dev)
    nb = 0
    n_full = idx.numel() // batch if (dev.type == "cuda" and engine.cfg.use_graph) else 0
    # EVAL_GROUP full batches per replay, as one forward of EVAL_GROUP x batch images:
    # with equal batch sizes the mean of the per-batch means is the mean over the group,
    # so the metric is unchanged; the larger forward runs the model at a better
    # fraction of the chip (the epoch-boundary evaluation: 64 ViT-tiny batches 19.4 ->
    # ~11 ms).  The remaining full batches and a ragged last one take the path below.
    G = EVAL_GROUP if n_full >= EVAL_GROUP else 1
    n_grp = n_full // G
    n_full = n_grp * G
    gb = G * batch
    if n_full:
        key = (pool.data_ptr(), gb, kind, total_steps, eval_rng.data_ptr())
        cache = engine.__dict__.setdefault("_eval_graphs", {})
        ent = cache.get(key)
        if ent is None:
            from ..utils.observe import drain_before_capture, is_capture_error, no_gc
            bidx = torch.zeros(gb, dtype=torch.int64, device=dev)
            acc = torch.zeros(1, dtype=torch.float64, device=dev)
            src = make_batcher(kind, pool, gb, eval_rng, total_steps, idx=bidx)
            saved = eval_rng.clone()
            bidx.copy_(idx[:gb].to(dev))
            s = torch.cuda.Stream(device=dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):  # warm-up (allocator, kernels)
                _eval_batch(prog, P, src, eval_rng, acc)
            torch.cuda.current_stream(dev).wait_stream(s)
            # same capture discipline as the step graphs (engine.CAPTURE_MODE): quiesce
            # (drain_before_capture), capture thread-local; if the CAPTURE fails,
            # evaluate eagerly for the rest of the run (same values, more launches) and
            # say why once; any other error propagates
            drain_before_capture(dev)
            g = torch.cuda.CUDAGraph()
            try:
                with no_gc(), torch.cuda.graph(g, capture_error_mode=CAPTURE_MODE):
                    _eval_batch(prog, P, src, eval_rng, acc)
                ent = (g, bidx, acc)
            except Exception as e:  # pragma: no cover - depends on the runtime
                if not is_capture_error(e):
                    raise
                import warnings
                warnings.warn(f"eval graph capture failed ({e!r}); evaluating eagerly for the rest of the run")
                torch.cuda.synchronize(dev)
                ent = (None, bidx, acc)
            eval_rng.copy_(saved)  # warm-up and capture leave the counters where they were
            cache[key] = ent
        g, bidx, acc = ent
        if g is not None:
            acc.zero_()
            for b in range(n_grp):
                bidx.copy_(idx[b * gb:(b + 1) * gb].to(dev), non_blocking=True)
                g.replay()
            total += acc * G  # each replay added the mean of its G batch means
            nb = n_full
        else:
            n_full = 0
    for s in range(n_full * batch, idx.numel(), batch):
        bidx_e = idx[s:s + batch].to(dev)
        src = make_batcher(kind, pool, bidx_e.numel(), eval_rng, total_steps, idx=bidx_e)
        _eval_batch(prog, P, src, eval_rng, total)
        nb += 1
    return float(total.item()) / max(nb, 1)


class _MicroCycle:
    """grad_accum > 1: the engine calls its batch source once per micro-batch, in
    order (also while capturing); call j of a step goes to micro-batch j's batcher,
    fused draw (``fused_spec``) included."""

    def __init__(self, batchers):
        self.batchers = batchers
        self.calls = 0

    def _next(self):
        b = self.batchers[self.calls % len(self.batchers)]
        self.calls += 1
        return b

    def __call__(self):
        return self._next()()

    def fused_spec(self):
        return self._next().fused_spec()


def train_worker(rank: int, world: int, cfg: ExperimentConfig, exp_name: str, paths: Paths,
                 local_rank: Optional[int] = None, backend: Optional[str] = None, verbose: bool = False) -> dict:
    local_rank = rank if local_rank is None else local_rank
    backend = backend or cfg.backend
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if world > 1:
        pdist.init_distributed(backend=backend, rank=rank, world_size=world)
    elif cfg.force_segments:
        pdist.init_single(backend=backend, device_index=local_rank)
    device = _device_for(rank, local_rank, backend)
    if device.type == "cuda":
        torch.cuda.set_device(device)
    torch.manual_seed(cfg.seed)

    train_pool, val_pool = _pools(cfg, device, rank)
    B = cfg.per_gpu_batch
    A = int(cfg.grad_accum)
    n_train, n_val = train_pool.shape[0], val_pool.shape[0]
    steps_per_epoch = len(shard_indices(n_train, world, rank, 0, cfg.seed)) // (B * A)
    if cfg.max_steps:
        steps_per_epoch = min(steps_per_epoch, cfg.max_steps)
    if steps_per_epoch < 1:
        raise ValueError(f"dataset too small: {n_train} images for batch {B} x {A} micro-batches x {world} ranks")
    val_idx0 = shard_indices(n_val, world, rank, 0, cfg.seed, shuffle=False, drop_last=False)
    val_batches = math.ceil(val_idx0.numel() / B)

    model = DiffusionVisionTransformer(**cfg.model_kwargs())
    init_path = os.path.join(paths.saved_dir, cfg.initializing)
    if rank == 0 and not os.path.isfile(init_path):
        ckpt.save_weights(model, init_path)
    pdist.barrier()
    ckpt.load_weights(model, init_path, strict=True)
    model.to(device).train()
    if rank == 0:
        printLog(f"Date: {asctime()}", paths.log)
        printLog("TrainSet batchs:" + str(steps_per_epoch), paths.log)
        printLog("TestSet batchs:" + str(val_batches), paths.log)

    temb_rows = int(math.log2(cfg.image_size[1])) + 1 if cfg.dataset.startswith("cold") else None
    ecfg = EngineConfig(lr=cfg.lr, t_max=steps_per_epoch * cfg.epoch[1], use_graph=cfg.graph,
                        bucket_blocks=cfg.bucket_blocks, seed=cfg.seed * 1000 + rank, temb_rows=temb_rows,
                        grad_accum=A, force_segments=cfg.force_segments, graph_steps=cfg.graph_steps)
    engine = TrainEngine(model, ecfg, device=device)
    # the epoch's DistributedSampler table [steps, micro-batch, B] lives on the device
    # (refilled once per epoch); the batch draw reads row ``scheduler step %
    # steps_per_epoch`` through the engine's device step counter, so replays need no
    # host copy per step and one hipGraph replay can run K whole steps.  The table is
    # rotated by the epoch's starting counter (one host read per epoch), so epoch e
    # reads its DistributedSampler batches in order even when the counter does not
    # start the epoch at a multiple of steps_per_epoch (a resume from a checkpoint of
    # another num_gpus / batch size / max_steps, or of the reference trainer).
    table_dev = torch.zeros(steps_per_epoch, A, B, dtype=torch.int64, device=device)
    batchers = [make_batcher(cfg.dataset, train_pool, B, engine.rng, cfg.model_total_steps, idx=table_dev,
                             idx_step=(engine.step_ctr[1:2], j * B)) for j in range(A)]
    engine.set_batch_fn(batchers[0] if A == 1 else _MicroCycle(batchers))

    start_epoch, end_epoch = int(cfg.epoch[0]), int(cfg.epoch[1])
    loss_rec, steps, best_loss = 5.0, 0, 5.0
    if cfg.resume and cfg.resume != "none":
        ck = ckpt.load_lastepoch(cfg.resume, model, engine)
        start_epoch = int(ck["epoch"]) + 1
        loss_rec = float(ck["loss_rec"])
        steps = int(ck["steps"])
        best_loss = float(ck["metric"])
        if rank == 0:
            printLog(f"resuming from epoch {start_epoch:8d} of " + cfg.resume, paths.log)
            printLog(f"recovering best_loss {best_loss:4f}", paths.log)
    engine.loss_ema.fill_(loss_rec)
    if cfg.comm_autotune and not cfg.comm_layout and engine.segmented and device.type == "cuda":
        times = engine.autotune_comm()  # training state restored afterwards
        if rank == 0 and times:
            printLog(f"# comm layout: {engine.comm_choice} " +
                     " ".join(f"{k}={v:.4f}ms" for k, v in times.items()), paths.log)
    if cfg.comm_layout and engine.segmented and device.type == "cuda":
        engine.apply_layout(cfg.comm_layout)
    check_param_sync(engine.flat_p, step=steps)  # replicas start identical
    writer = ScalarWriter(paths.ckpt_dir, enabled=(rank == 0))
    clock = StepClock(device)
    clock.mark(steps)
    prof = torch_profiler(rank)
    if prof is not None:
        prof.__enter__()
    # eval draws (cold t per sample): independent per rank, like each rank's DataLoader
    # in the reference; the counter is derived from the epoch, so a resumed run
    # evaluates epoch e with the same draws as an uninterrupted one
    eval_rng = torch.tensor([cfg.seed + 7919 + 1000003 * rank, 0], dtype=torch.int64, device=device)

    history = []
    last_ms = None  # device ms/step of the last full log window
    ckw = ckpt.CheckpointWriter()
    if rank == 0:
        ckw.warm()
        # the first torch optimizer / scheduler built in a process imports the compiler stack
        # (~1.5 s): pay it here, not inside the first background checkpoint write
        engine.scheduler_state_dict()
        engine._optimizer_sd(engine.flat_m, engine.flat_v, 0, 0)
    t_start = time.time()
    t_run = t_epoch = time.perf_counter()
    steps0 = steps
    try:
        for epoch in range(start_epoch, end_epoch):
            model.train()
            table = shard_indices(n_train, world, rank, epoch, cfg.seed)[: steps_per_epoch * A * B]
            base = int(engine.step_ctr[1].item()) % steps_per_epoch  # the row this epoch's first step reads
            table_dev.copy_(table.view(steps_per_epoch, A, B).roll(base, 0))
            s = 0
            while s < steps_per_epoch:
                # run up to the next point the host must act at (log line, sync check,
                # injected fault, epoch end): whole K-step graph replays in between
                n = steps_per_epoch - s
                n = min(n, cfg.log_every - steps % cfg.log_every)
                if cfg.sync_check_every:
                    n = min(n, cfg.sync_check_every - steps % cfg.sync_check_every)
                if cfg.fault_inject_step and steps < cfg.fault_inject_step:
                    n = min(n, cfg.fault_inject_step - steps)
                if prof is not None:
                    n = 1
                with phase("train_steps"):
                    engine.train_steps(n, materialize=False)  # lazy time_embed decay: applied at the epoch end
                if prof is not None:
                    prof.step()
                steps += n
                s += n
                if cfg.sync_check_every and steps % cfg.sync_check_every == 0:
                    check_param_sync(engine.flat_p, step=steps)
                if steps % cfg.log_every == 0:
                    window = clock.mark(steps)  # device events: the only sync of the window
                    if window is not None and window[1] > 0:
                        last_ms = 1e3 * window[0] / window[1]
                    engine.check_comm()  # a timed-out bucket hand-off stops the run (stale gradients)
                    loss_rec = float(engine.loss_ema.item())
                    if verbose:
                        print(f"[rank {rank}] step {steps} loss_ema {loss_rec:.4f}", flush=True)
                    if rank == 0:
                        now = time.time()
                        printLog(fmt_steps(steps, loss_rec, now - t_start), paths.log)
                        t_start = now
                        if cfg.perf_log and window is not None and window[1] > 0:
                            sec, n = window
                            printLog(f"# perf: {n * B * A * world / sec:.1f} img/s  {1e3 * sec / n:.3f} ms/step "
                                     f"(device, {world} rank(s)" +
                                     (f", comm {engine.comm_choice or 'default'}/{engine.handoff_order}"
                                      if engine.segmented else "") + ")", paths.log)
                if cfg.fault_inject_step and steps >= cfg.fault_inject_step and cfg.fault_inject_rank in (-1, rank):
                    raise FaultInjected(f"fault injected at step {steps} on rank {rank} (fault_inject_step)")
            engine.materialize_lazy()
            loss_rec = float(engine.loss_ema.item())
            engine.check_comm()  # epoch end: before evaluating / checkpointing these weights
            t_ev = time.perf_counter()
            if (epoch - start_epoch + 1) % max(cfg.eval_every, 1) == 0 or epoch == end_epoch - 1:
                model.eval()
                vidx = shard_indices(n_val, world, rank, epoch, cfg.seed, shuffle=False, drop_last=False)
                eval_rng[1] = epoch * val_batches
                with phase("evaluate"):
                    vloss = evaluate(model, engine, val_pool, vidx, B, cfg.dataset, cfg.model_total_steps, eval_rng)
                vloss = pdist.all_reduce_mean(vloss, device)
                model.train()
                history.append((epoch, vloss))
                t_ck = time.perf_counter()
                if rank == 0:
                    printLog(fmt_epoch(epoch, vloss), paths.log)
                    writer.add_scalar("loss", vloss, epoch)
                    best = vloss < best_loss
                    if best:
                        best_loss = vloss
                    # bestloss.pkl / lastepoch.pkl written by a background thread from a
                    # snapshot taken here (device copies on the training stream, host copy
                    # on a side stream) while the next epoch trains; the writer takes the
                    # snapshot only once the previous write has released its buffers
                    ckw.submit(engine.snapshot_to_host, os.path.join(paths.ckpt_dir, "lastepoch.pkl"), epoch,
                               steps, loss_rec, best_loss,
                               best_path=os.path.join(paths.ckpt_dir, "bestloss.pkl") if best else None)
                pdist.barrier()
                t_end = time.perf_counter()
                if rank == 0 and cfg.perf_log:
                    wall = t_end - t_epoch
                    printLog(f"# perf: epoch {epoch} end to end {steps_per_epoch * B * A * world / wall:.1f} img/s "
                             f"({wall:.3f} s: evaluate {1e3 * (t_ck - t_ev):.1f} ms, checkpoint hand-off "
                             f"{1e3 * (t_end - t_ck):.1f} ms, previous write {1e3 * ckw.last_write_s:.1f} ms "
                             f"in the background: host copy wait {1e3 * ckw.last_write_parts[0]:.1f}, layout "
                             f"{1e3 * ckw.last_write_parts[1]:.1f}, files {1e3 * ckw.last_write_parts[2]:.1f})",
                             paths.log)
            t_epoch = time.perf_counter()
    except BaseException:
        # a failing step (or an injected fault) must not cut the previous epoch's
        # background checkpoint write short: the resume reads those files
        try:
            ckw.join()
        except RuntimeError as werr:
            print(f"[rank {rank}] {werr}", flush=True)
        raise
    if prof is not None:
        prof.__exit__(None, None, None)
    t_done = time.perf_counter()
    ckw.join()  # the last epoch's files are complete before the run returns
    writer.close()
    e2e = (steps - steps0) * B * A * world / max(t_done - t_run, 1e-9)
    if rank == 0 and cfg.perf_log and steps > steps0:
        printLog(f"# perf: run end to end {e2e:.1f} img/s over {steps - steps0} steps "
                 f"({t_done - t_run:.2f} s incl. graph capture, evaluation, checkpoints)", paths.log)
    result = {"steps": steps, "loss_rec": loss_rec, "best_loss": best_loss, "history": history,
              "e2e_img_per_s": e2e,
              "final_lr": engine.current_lr(), "rng": [int(v) for v in engine.rng.tolist()],
              "eval_rng": [int(v) for v in eval_rng.tolist()],
              "comm_choice": engine.comm_choice, "handoff_order": engine.handoff_order,
              "ms_per_step": last_ms}
    engine.close()
    pdist.cleanup()
    return result


def _spawn_entry(rank, world, cfg, exp_name, paths, backend, port, queue):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["RANK"] = str(rank)
    os.environ["WORLD_SIZE"] = str(world)
    os.environ["LOCAL_RANK"] = str(rank)
    res = train_worker(rank, world, cfg, exp_name, paths, local_rank=rank, backend=backend)
    if queue is not None:
        queue.put((rank, res))


def launch(cfg: ExperimentConfig, exp_name: str, paths: Paths, backend: Optional[str] = None) -> dict:
    """Run the experiment: torchrun env -> this rank; num_gpus == 1 -> in-process;
    else spawn one process per rank and fail fast if any exits non-zero
    (the reference ``join``-ed without checking exit codes)."""
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ:
        w, r, l = pdist.env_world()
        return train_worker(r, w, cfg, exp_name, paths, local_rank=l, backend=backend)
    world = int(cfg.num_gpus)
    if world <= 1:
        return train_worker(0, 1, cfg, exp_name, paths, backend=backend)
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    port = pdist.free_port()
    q = ctx.Queue()
    procs = [ctx.Process(target=_spawn_entry, args=(r, world, cfg, exp_name, paths, backend, port, q),
                         name=f"rank{r}") for r in range(world)]
    for p in procs:
        p.start()
    # drain the result queue WHILE the ranks run: a child cannot exit before its
    # queued result has been flushed into the pipe, so joining first could deadlock
    import queue as _queue
    per_rank = {}
    while True:
        got = False
        try:
            r, res = q.get(timeout=0.5)
            per_rank[r] = res
            got = True
        except _queue.Empty:
            pass
        failed = [p for p in procs if p.exitcode not in (None, 0)]
        if failed:
            # every rank that has failed by now (the first to die usually takes its
            # peers' collectives down with it), then stop the rest
            msg = ", ".join(f"{p.name} (exit {p.exitcode})" for p in failed)
            for p in procs:
                if p.is_alive():
                    p.terminate()
            for p in procs:
                p.join()
            raise RuntimeError(f"rank process(es) failed: {msg}")
        if len(per_rank) == world or (not got and not any(p.is_alive() for p in procs)):
            break
    for p in procs:
        p.join()
    bad = [p.exitcode for p in procs if p.exitcode != 0]
    if bad:
        raise RuntimeError(f"rank processes failed with exit codes {bad}")
    if len(per_rank) != world:
        raise RuntimeError(f"only ranks {sorted(per_rank)} of {world} reported a result")
    out = dict(per_rank.get(0, {}))
    out["per_rank"] = per_rank  # every rank's result (rank 0's is also the top level)
    return out
