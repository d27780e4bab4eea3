#!/usr/bin/env python3
"""Headline benchmark: train img/s (whole node), ViT-tiny 64x64 cold diffusion.

Config = the reference's measured run (20220822.yaml, ViT-tiny
D=384 depth 7 12 heads p=8, per-GPU batch 32 = batch_size 16 x2 (AMP),
AdamW wd 0.05 + clip 1.0 + cosine LR, smooth-L1, cold pixelation task), on
synthetic Oxford-Flowers-shaped images generated on the device and
random-init weights (no datasets / checkpoints available offline).
Weak scaling: per-GPU batch fixed at 32, N ranks, data parallel over RCCL.

Timed region: exactly K full optimizer steps (on-device batch draw + forward +
loss + backward + bucketed all-reduce + clip + AdamW + LR schedule), bracketed
by barrier + synchronize on both sides; max over ranks.  Also reports (extra
keys, rank 0, outside the timed region) the DDIM k=20 / N=64 sampler
throughput of the hipGraph-captured sampling loop.

    python bench.py                       # 1 GPU
    python bench.py --gpus N              # N ranks, spawned here (one process per GPU)
    torchrun --nproc-per-node N bench.py --gpus N --steps K --warmup W

``--gpus N`` is honoured either way: under torchrun the launched world size must
equal N (else exit 2); without torchrun env vars and N > 1 this process spawns
N rank processes itself (multi_gpu_trainer.py:212-219 launches its ranks the same
way) without touching the GPU, and exits with the first non-zero rank exit code.
"""
import time

_T_START = time.time()  # process start: the rank deadline counts the interpreter / torch import too

import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch
import torch.distributed as dist

# rehearsal of the multi-rank flow on a 1-GPU box: every rank on device 0 over gloo
# (RCCL refuses two ranks on one device); timings are NOT a scaling measurement
SHARED_GPU = os.environ.get("DDIM_COLD_REHEARSE_SHARED_GPU") == "1"
BASELINE_IMG_S_PER_GPU = 709.0  # 22.2 steps/s x 32 img (train.log, RTX 3090 fp16 AMP)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--model", default="vit_tiny")
    ap.add_argument("--batch", type=int, default=32, help="per-GPU batch (yaml batch_size 16 x2 for AMP)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--graph-steps", type=int, default=4,
                    help="optimizer steps per hipGraph replay (TrainEngine.train_steps; every step fully executed)")
    ap.add_argument("--graph-warmup", type=int, default=1,
                    help="eager steps before the graphs are captured (EngineConfig.graph_warmup): with 1, the "
                         "rest of the --warmup steps replay the captured K-step graph, so the timed steps start "
                         "on a graph that has run and a device that is busy (profiles/first_replay_r6.txt)")
    ap.add_argument("--bucket-blocks", type=int, default=2)
    ap.add_argument("--no-sampler", action="store_true")
    ap.add_argument("--force-dist", action="store_true",
                    help="init the RCCL process group and run segmented graphs + collectives even with 1 rank")
    ap.add_argument("--segmented-comm", action="store_true",
                    help="host-issued all-reduces between graph segments instead of capturing them in the step graph")
    ap.add_argument("--captured-comm", action="store_true",
                    help="capture the collectives in the step graph (a comm-stream branch) instead of issuing them "
                         "from the host between the event-split step graphs (the default)")
    ap.add_argument("--grad-wire", default="fp32", choices=["fp32", "bf16"],
                    help="gradient all-reduce wire format (bf16 halves the xGMI bytes)")
    ap.add_argument("--comm", default="auto", choices=["auto", "torch", "native"],
                    help="gradient collectives through torch.distributed (RCCL) or the native RCCL communicator "
                         "(auto: native if it comes up and verifies on every rank)")
    ap.add_argument("--comm-layout", default="auto",
                    help="data parallel: gradient-exchange layout (overlap-<blocks per bucket> | inline-1); auto = "
                         "TrainEngine.autotune_comm() measures the cost model's pick + overlap-2/4 + inline-1 on this "
                         "job's ranks before the warmup (training state restored afterwards)")
    ap.add_argument("--sampler-k", type=int, default=20)
    ap.add_argument("--sampler-n", type=int, default=64)
    ap.add_argument("--sampler-host-noise", action="store_true",
                    help="draw the sampler's x_T on the host (torch.normal on CPU, as the reference)")
    ap.add_argument("--dataset", default="cold", choices=["cold", "gaussian"],
                    help="training task of the timed steps: cold pixelation pairs (the reference's measured "
                         "run) or Gaussian DDIM (diffusion_loader.DiffusionDataset: q_sample, t in 0..1999)")
    ap.add_argument("--no-gaussian", action="store_true",
                    help="1 GPU: skip the extra Gaussian-DDIM training throughput key")
    ap.add_argument("--no-hires", action="store_true",
                    help="1 GPU: skip the extra vit_small_200 (200x200, BASELINE.json config 4) and "
                         "oxford_flower training keys")
    ap.add_argument("--no-eager-baseline", action="store_true",
                    help="skip timing the plain eager PyTorch sampler (BASELINE.md's sampling comparator)")
    ap.add_argument("--no-vendor", action="store_true",
                    help="1 GPU: skip the same-node vendor comparators (stock PyTorch-ROCm ops: hipBLASLt, SDPA, "
                         "fused AdamW; training step and DDIM sampler each captured whole in one graph)")
    return ap.parse_args(argv)


# Bounds that keep a hung multi-GPU run diagnosable inside the driver's 600 s limit
# (ddim_cold_amd/parallel/watchdog.py): the process-group timeout, every rank's own
# deadline (prints all ranks' last phases, then exits) and the self-spawning parent's.
PG_TIMEOUT_S = int(os.environ.get("DDIM_COLD_PG_TIMEOUT_S", "120"))
RANK_DEADLINE_S = float(os.environ.get("DDIM_COLD_DEADLINE_S", "450"))
SPAWN_DEADLINE_S = float(os.environ.get("DDIM_COLD_SPAWN_DEADLINE_S", str(RANK_DEADLINE_S + 30)))


def _rank_entry(rank: int, world: int, port: int, argv, phase_dir: str):
    """Spawned rank process (self-launch): torchrun-style env, then the benchmark."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world), DDIM_COLD_PHASE_DIR=phase_dir)
    run(parse_args(argv))


def spawn_ranks(n: int, argv, deadline_s: float = None) -> int:
    """Launch ``n`` rank processes of this benchmark (spawn context) and wait; on the
    first non-zero exit the others are terminated.  The parent never initialises the
    GPU (only counts devices), so the children own it.  A wall-clock deadline
    (``DDIM_COLD_SPAWN_DEADLINE_S``) bounds the whole launch: when it passes, the
    parent prints every rank's last phase (watchdog.report_dir), terminates the
    ranks and returns 124.  Returns the exit code."""
    import multiprocessing as mp
    import shutil
    import tempfile
    from ddim_cold_amd.parallel.dist import free_port
    from ddim_cold_amd.parallel.watchdog import report_dir
    deadline_s = SPAWN_DEADLINE_S if deadline_s is None else deadline_s
    ndev = torch.cuda.device_count()  # no HIP context is created by counting
    if 0 < ndev < n and not SHARED_GPU:
        print(f"bench.py: --gpus {n} but only {ndev} GPU(s) visible", file=sys.stderr)
        return 2
    ctx = mp.get_context("spawn")
    port = free_port()
    phase_dir = tempfile.mkdtemp(prefix="ddim_cold_phases_")
    t0 = time.time()
    procs = [ctx.Process(target=_rank_entry, args=(r, n, port, argv, phase_dir), name=f"rank{r}")
             for r in range(n)]
    for p in procs:
        p.start()
    code = 0
    try:
        while any(p.is_alive() for p in procs):
            for p in procs:
                p.join(timeout=0.2)
                if p.exitcode not in (None, 0) and code == 0:
                    code = p.exitcode if p.exitcode > 0 else 1
                    print(f"bench.py: {p.name} exited with code {p.exitcode}; stopping the other ranks\n"
                          f"{report_dir(phase_dir, n, since=t0)}", file=sys.stderr, flush=True)
                    for q in procs:
                        if q.is_alive():
                            q.terminate()
            if code == 0 and time.time() - t0 > deadline_s:
                code = 124
                print(f"bench.py: launch deadline of {deadline_s:.0f}s passed; terminating the ranks\n"
                      f"{report_dir(phase_dir, n, since=t0)}", file=sys.stderr, flush=True)
                for q in procs:
                    if q.is_alive():
                        q.terminate()
                t_kill = time.time() + 10
                for q in procs:
                    q.join(timeout=max(0.1, t_kill - time.time()))
                    if q.is_alive():
                        q.kill()
        for p in procs:
            p.join()
            if p.exitcode not in (0, None) and code == 0:
                code = p.exitcode if p.exitcode > 0 else 1
    finally:
        shutil.rmtree(phase_dir, ignore_errors=True)
    return code


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse_args(argv)
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" in os.environ:  # launched by torchrun (or another env launcher)
        world = int(os.environ["WORLD_SIZE"])
        if world != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks",
                  file=sys.stderr)
            raise SystemExit(2)
        run(args)
        return 0
    if args.gpus > 1:
        raise SystemExit(spawn_ranks(args.gpus, argv))
    run(args)
    return 0


def _time_train(args, name, dataset, dev, lr, seed, prefix, pool=None):
    """One extra 1-GPU training measurement outside the headline number: model
    ``name`` on the ``dataset`` task at the headline's per-GPU batch, optimizer and
    graph settings, ``--warmup`` untimed then exactly ``--steps`` timed steps between
    synchronizes.  Returns ``{prefix_img_per_s, prefix_ms_per_step, prefix_final_loss}``."""
    from ddim_cold_amd.models import build_model
    from ddim_cold_amd.train.engine import EngineConfig, TrainEngine
    from ddim_cold_amd.data.synthetic import ColdBatcher, GaussianBatcher, synthetic_pool
    torch.manual_seed(1234)
    m = build_model(name).to(dev).train()
    if pool is None or tuple(pool.shape[-2:]) != tuple(m.img_size):
        pool = synthetic_pool(1024, tuple(m.img_size), seed=7, device=dev)
    cold = dataset == "cold"
    e = TrainEngine(m, EngineConfig(lr=lr, t_max=512 * 100, use_graph=not args.no_graph, seed=seed,
                                    temb_rows=int(math.log2(m.img_size[1])) + 1 if cold else None,
                                    graph_steps=args.graph_steps, graph_warmup=args.graph_warmup), device=dev)
    e.set_batch_fn(ColdBatcher(pool, args.batch, e.rng) if cold else
                   GaussianBatcher(pool, args.batch, e.rng, m.total_steps))
    e.train_steps(args.warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e.train_steps(args.steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    loss = float(e.loss_last.item())
    if not math.isfinite(loss):
        raise SystemExit(f"non-finite {prefix} loss {loss}")
    e.close()
    del e, m, pool
    torch.cuda.empty_cache()
    return {f"{prefix}_img_per_s": round(args.batch * args.steps / dt, 1),
            f"{prefix}_ms_per_step": round(dt / args.steps * 1e3, 4),
            f"{prefix}_final_loss": round(loss, 5)}


def run(args):
    from ddim_cold_amd.parallel.dist import (init_distributed, init_single, all_reduce_max, barrier, cleanup,
                                             env_world)
    from ddim_cold_amd.parallel import watchdog
    from ddim_cold_amd.parallel.watchdog import phase
    world, rank, local = env_world()
    if SHARED_GPU:
        local = 0
    # per-rank phase markers on stderr + a deadline that names every rank's last phase
    watchdog.install(rank, world, deadline_s=RANK_DEADLINE_S, since=_T_START)
    phase("pg-init", world=world, timeout_s=PG_TIMEOUT_S)
    if args.force_dist and world == 1:
        distributed = init_single(device_index=local, timeout_s=PG_TIMEOUT_S)
    else:
        distributed = init_distributed(backend="gloo" if SHARED_GPU else None, timeout_s=PG_TIMEOUT_S)
    phase("pg-ready", backend=dist.get_backend() if dist.is_initialized() else "none")
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    n = dist.get_world_size() if dist.is_initialized() else 1
    if n != args.gpus and not (args.force_dist and n == 1):
        raise SystemExit(f"bench.py: process group has {n} ranks, --gpus {args.gpus}")

    from ddim_cold_amd.models import build_model
    from ddim_cold_amd.train.engine import EngineConfig, TrainEngine
    from ddim_cold_amd.data.synthetic import ColdBatcher, GaussianBatcher, synthetic_pool

    torch.manual_seed(1234)
    model = build_model(args.model).to(dev).train()
    base_lr = 0.005
    lr = base_lr * args.batch * n / 512  # multi_gpu_trainer.py:196
    cfg = EngineConfig(lr=lr, t_max=512 * 100, use_graph=not args.no_graph, bucket_blocks=args.bucket_blocks,
                       seed=42, force_segments=args.force_dist,
                       # cold t in 1..log2(W); Gaussian t spans the whole table
                       temb_rows=int(math.log2(model.img_size[1])) + 1 if args.dataset == "cold" else None,
                       graph_comm=not args.segmented_comm, grad_wire=args.grad_wire,
                       comm_events=not (args.segmented_comm or args.captured_comm),
                       comm="torch" if SHARED_GPU else args.comm, graph_steps=args.graph_steps,
                       graph_warmup=args.graph_warmup)
    phase("engine-build", model=args.model)
    engine = TrainEngine(model, cfg, device=dev)
    phase("engine-ready", comm=engine.comm_backend if engine.segmented else "none")
    pool = synthetic_pool(1024, tuple(model.img_size), seed=7 + rank, device=dev)
    if args.dataset == "cold":
        engine.set_batch_fn(ColdBatcher(pool, args.batch, engine.rng))
    else:
        engine.set_batch_fn(GaussianBatcher(pool, args.batch, engine.rng, model.total_steps))

    comm_model = None
    if engine.segmented and dev.type == "cuda":
        # outside the timed region; parameters / moments / counters / RNG restored
        if n > 1:
            # measured all-reduce curve on this job's ranks -> fitted cost model, which
            # orders the bucket layouts (parallel/costmodel.py); outside the timed region
            phase("probe-allreduce")
            try:
                fit, probe = engine.probe_allreduce()
                comm_model = {"probe_us": {f"{b / 2**20:g}MB": round(u, 1) for b, u in probe.items()},
                              "alpha_us": round(fit.alpha_us, 2), "algbw_GBs": round(fit.algbw_gbs, 1),
                              "busbw_GBs": round(fit.busbw_gbs, 1),
                              "predicted_exposed_us": {L[0]: round(L[4], 1) for L in engine.model_layouts()[:4]}}
            except Exception as e:  # diagnostics only: the benchmark goes on with the fixed candidates
                comm_model = {"error": repr(e)[:200]}
                engine.comm_fit = None
        if args.comm_layout == "auto":
            phase("autotune")
            engine.autotune_comm()
        else:
            engine.apply_layout(args.comm_layout)
    phase("warmup", steps=args.warmup, layout=engine.comm_choice)
    engine.train_steps(args.warmup)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    phase("timed", steps=args.steps)
    t0 = time.perf_counter()
    engine.train_steps(args.steps)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    phase("timed-done", ms_per_step=round(elapsed / args.steps * 1e3, 4))
    elapsed = all_reduce_max(elapsed, dev)
    engine.check_comm()
    loss = float(engine.loss_last.item())
    if not math.isfinite(loss):
        raise SystemExit(f"non-finite loss {loss}")

    ms = elapsed / args.steps * 1e3
    value = n * args.batch * args.steps / elapsed
    extra = {}
    if rank == 0 and n == 1 and args.dataset == "cold" and not args.no_gaussian and dev.type == "cuda":
        # the reference's other training task (DiffusionDataset, diffusion_loader.py:24-58):
        # Gaussian DDIM, q_sample batch drawn inside the patch-embedding launch, same
        # model / batch / optimizer; timed the same way (outside the headline number)
        phase("extra:gaussian-ddim")
        extra.update(_time_train(args, args.model, "gaussian", dev, lr, seed=43, pool=pool,
                                 prefix="gaussian_ddim_train"))
    if rank == 0 and n == 1 and args.dataset == "cold" and args.model == "vit_tiny" and not args.no_hires \
            and dev.type == "cuda":
        # BASELINE.json config 4 (the 200x200 high-resolution path) and the
        # sampling CLI's oxford_flower model (ViT.py:277), trained the same way as the
        # headline: same per-GPU batch, full AdamW step, K-step graphs, timed between
        # synchronizes over exactly --steps steps after --warmup (1 GPU; the scaling
        # curve is the headline model's)
        for name, key in (("vit_small_200", "vit_small_200_train"), ("oxford_flower", "oxford_flower_train")):
            phase(f"extra:{name}")
            extra.update(_time_train(args, name, "cold", dev, lr, seed=44, prefix=key))
    if rank == 0 and n == 1 and args.dataset == "cold" and not args.no_vendor and dev.type == "cuda":
        # same-node vendor comparator: the reference step (multi_gpu_trainer.py:115-134) from stock
        # PyTorch-ROCm ops (hipBLASLt / SDPA / fused AdamW), captured whole in one graph
        from ddim_cold_amd.bench.vendor_baseline import time_vendor_train
        torch.manual_seed(1234)
        vm = build_model(args.model).to(dev).train()
        vdt, vloss, vkind = time_vendor_train(vm, pool, args.batch, lr, 512 * 100, steps=args.steps,
                                              warmup=args.warmup)
        extra["train_vendor_graph_img_per_s"] = round(args.batch / vdt, 1)
        extra["train_vendor_graph_ms_per_step"] = round(vdt * 1e3, 4)
        extra["train_vs_vendor_graph"] = round((value / n) / (args.batch / vdt), 2)
        extra["train_vendor_config"] = {"attn": "sdpa", "optimizer": f"AdamW({vkind})", "graph": True,
                                        "autocast": "bf16", "final_loss": round(vloss, 5)}
        del vm
    # the sampler metric is a 1-GPU number (BASELINE.json config 5): multi-rank runs skip it
    if rank == 0 and n == 1 and not args.no_sampler and dev.type == "cuda":
        from ddim_cold_amd.diffusion.samplers import DDIMSampler
        model.eval()
        s = DDIMSampler(model, dev, k=args.sampler_k)
        # x_T drawn on the device (seeded); --sampler-host-noise: on the host as the reference
        g = torch.Generator(device=dev if not args.sampler_host_noise else "cpu").manual_seed(0)
        dn = not args.sampler_host_noise
        s.sample(args.sampler_n, generator=g, device_noise=dn)  # capture
        torch.cuda.synchronize()
        reps = 10
        ts = time.perf_counter()
        for _ in range(reps):  # every batch: noise draw, the 100-step graph, result copied to the host
            s.sample(args.sampler_n, generator=g, device_noise=dn)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - ts) / reps
        extra.update({"ddim_sampler_img_per_s": round(args.sampler_n / dt, 1),
                      "ddim_sampler_ms_per_batch": round(dt * 1e3, 3),
                      "ddim_sampler_config": {"k": args.sampler_k, "N": args.sampler_n, "steps": len(s.ts),
                                              "graph": True, "noise": "device" if dn else "host"}})
        if not args.no_eager_baseline:
            # the sampling yardstick is a plain eager PyTorch-ROCm
            # implementation of the same math on the same GPU (fp32, as the
            # reference samples; bf16-autocast variant reported too)
            from ddim_cold_amd.bench.eager_sampler import time_eager_sampler
            e32 = time_eager_sampler(model, dev, args.sampler_k, args.sampler_n, device_noise=dn)
            ebf = time_eager_sampler(model, dev, args.sampler_k, args.sampler_n, autocast_bf16=True, device_noise=dn)
            extra["ddim_sampler_eager_torch_fp32_img_per_s"] = round(args.sampler_n / e32, 1)
            extra["ddim_sampler_eager_torch_bf16_img_per_s"] = round(args.sampler_n / ebf, 1)
            extra["ddim_sampler_vs_eager_fp32"] = round(e32 / dt, 2)
        if not args.no_vendor:
            # same-node vendor comparator: the 100-step loop from stock ops (SDPA, hipBLASLt,
            # bf16 autocast, fp32 update) unrolled into one graph
            from ddim_cold_amd.bench.vendor_baseline import time_vendor_sampler
            vs = time_vendor_sampler(model, args.sampler_n, args.sampler_k, reps=5)
            extra["ddim_sampler_vendor_graph_img_per_s"] = round(args.sampler_n / vs, 1)
            extra["ddim_sampler_vs_vendor_graph"] = round(vs / dt, 2)
        # BASELINE.json config 5, second half: the draft->drawing img2img call of
        # ViT_draft2drawing.py:389-409 (9 t_starts 1599..1999, k=10, up to 200 steps)
        # as ONE batched replayed hipGraph; comparator = the reference's sequential
        # batch-1 fp32 eager loop on the same GPU
        from ddim_cold_amd.bench.eager_sampler import time_img2img
        starts = list(range(1599, 2000, 50))
        ti = time_img2img(model, dev, starts, 10, reps=10)
        extra["draft2drawing_ms"] = round(ti * 1e3, 3)
        extra["draft2drawing_img_per_s"] = round(len(starts) / ti, 1)
        if not args.no_eager_baseline:
            te = time_img2img(model, dev, starts, 10, eager=True)
            extra["draft2drawing_eager_torch_fp32_ms"] = round(te * 1e3, 1)
            extra["draft2drawing_vs_eager_fp32"] = round(te / ti, 2)
        if not args.no_vendor:
            # same batching (9 starts in one batch on the shared grid) and one graph, stock
            # ops: the kernel-quality comparator of the img2img path
            from ddim_cold_amd.bench.vendor_baseline import time_vendor_img2img
            tv = time_vendor_img2img(model, starts, 10, reps=5)
            extra["draft2drawing_vendor_graph_ms"] = round(tv * 1e3, 3)
            extra["draft2drawing_vs_vendor_graph"] = round(tv / ti, 2)
        model.train()
    if rank == 0:
        out = {
            "metric": ("train imgs/sec (whole node) ViT-tiny 64x64" if args.model == "vit_tiny"
                       else f"train imgs/sec (whole node) {args.model}") +
                      ("" if args.dataset == "cold" else " Gaussian DDIM"),
            "value": round(value, 1),
            "unit": "img/s",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            # the reference's number is for the vit_tiny yaml config only
            "vs_baseline": round(value / (BASELINE_IMG_S_PER_GPU * n), 3)
                           if args.model == "vit_tiny" and args.dataset == "cold" else None,
            "dtype": "bf16",
            "data": "synthetic (on-device Oxford-Flowers-shaped pool, " +
                    ("cold pixelation pairs" if args.dataset == "cold" else "Gaussian DDIM q_sample pairs") +
                    "), random-init weights",
            "config": {"model": f"{args.model} (D={model.embed_dim}, depth={len(model.blocks)}, "
                                f"heads={model.blocks[0].attn.num_heads}, patch={model.patch_size}, "
                                f"{model.img_size[0]}x{model.img_size[1]})", "global_batch": args.batch * n,
                       "per_gpu_batch": args.batch, "seq_len": model.num_tokens, "parallelism": f"dp{n}",
                       "graph": bool(engine.cfg.use_graph),
                       # event-split data parallel: two graphs per step, collectives between
                       "graph_steps": args.graph_steps if not (engine.segmented and engine.cfg.comm_events) else 1,
                       "graph_warmup": engine.cfg.graph_warmup,
                       "bucket_blocks": engine.cfg.bucket_blocks if engine.segmented else None,
                       "allreduce": ("none" if not engine.segmented else "eager" if dev.type != "cuda" else
                                     "eager-inline-fallback" if engine.comm_fallback else
                                     "host-issued-between-event-split-graphs" if engine.cfg.comm_events else
                                     "segmented" if (args.segmented_comm or getattr(engine, "_graph_comm_failed", False))
                                     else "captured-in-graph-inline" if engine.cfg.comm_inline
                                     else "captured-in-graph-comm-branch"),
                       "autotune_s": round(getattr(engine, "autotune_s", 0.0), 2) or None,
                       "autotune_dropped": getattr(engine, "autotune_errors", None) or None,
                       "grad_wire": args.grad_wire,
                       "comm": engine.comm_backend if engine.segmented else "none",
                       "native_comm_error": engine.native_error,
                       "comm_fallback": engine.comm_fallback,
                       "comm_layout": engine.comm_choice,
                       "handoff": engine.handoff_order,
                       "rccl_ranks": engine.ncomm.info()[0] if engine.ncomm is not None else
                       (n if distributed and dist.get_backend() == "nccl" else None),
                       "launcher": "torchrun/env" if os.environ.get("TORCHELASTIC_RUN_ID") else
                       ("self-spawn" if n > 1 else "single"),
                       "comm_layout_ms": {k: round(v, 4) for k, v in engine.comm_times.items()} or None,
                       "comm_model": comm_model,
                       "optimizer": "AdamW(wd=0.05)+clip1.0+cosine", "final_loss": round(loss, 5)},
        }
        out.update(extra)
        if SHARED_GPU:  # not a scaling measurement: every rank on device 0 over gloo
            out["rehearsal_shared_gpu_gloo"] = True
        print(json.dumps(out), flush=True)
    phase("teardown")
    engine.close()
    cleanup()
    phase("done")


if __name__ == "__main__":
    main()
