"""Host-side timing of the event-split data-parallel step (1-rank group on one GPU):
how long the host spends in each call of ``TrainEngine._replay`` (compute-graph
replay, the per-bucket comm-stream issue, the join, the optimizer-graph replay).
If a graph replay blocks the host until the GPU finishes it, the comm-stream work
can only be issued after the whole backward and nothing overlaps.

    python tools/host_timing.py [--layout overlap-2]   (DDIM_COLD_FAKE_COMM=1 optional)
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.distributed as dist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layout", default="overlap-2")
    ap.add_argument("--steps", type=int, default=200)
    args = ap.parse_args()
    from ddim_cold_amd.parallel.dist import free_port, graph_safe_nccl_env
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(free_port()))
    graph_safe_nccl_env()
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from ddim_cold_amd.models import build_model
    from ddim_cold_amd.train.engine import EngineConfig, TrainEngine
    from ddim_cold_amd.data.synthetic import ColdBatcher, synthetic_pool
    torch.manual_seed(0)
    model = build_model("vit_tiny").cuda().train()
    eng = TrainEngine(model, EngineConfig(lr=1e-4, t_max=1000, force_segments=True, temb_rows=7))
    eng.set_batch_fn(ColdBatcher(synthetic_pool(256, device="cuda"), 32, eng.rng))
    L = {l[0]: l for l in eng.COMM_LAYOUTS}[args.layout]
    eng.set_comm_layout(L[1], L[2], L[3])
    eng.train_steps(20)
    torch.cuda.synchronize()
    g1, g2 = eng._graphs
    evs = eng._events
    acc = {"g1.replay": 0.0, "issue": 0.0, "join": 0.0, "g2.replay": 0.0}
    t_start = time.perf_counter()
    for _ in range(args.steps):
        t0 = time.perf_counter()
        g1.replay()
        t1 = time.perf_counter()
        sig = eng._signal
        if sig is not None:
            sig.expected += 1
        for k, ev in enumerate(evs):
            eng._allreduce(k, after=ev)
        t2 = time.perf_counter()
        eng._join_comm()
        t3 = time.perf_counter()
        g2.replay()
        t4 = time.perf_counter()
        eng.steps_done += 1
        acc["g1.replay"] += t1 - t0
        acc["issue"] += t2 - t1
        acc["join"] += t3 - t2
        acc["g2.replay"] += t4 - t3
    host = time.perf_counter() - t_start
    torch.cuda.synchronize()
    wall = time.perf_counter() - t_start
    n = args.steps
    print(f"layout {args.layout} signal {eng.cfg.comm_signal} fake={os.environ.get('DDIM_COLD_FAKE_COMM', '0')}: "
          + " ".join(f"{k}={v / n * 1e6:.1f}us" for k, v in acc.items())
          + f" host/step={host / n * 1e6:.1f}us wall/step={wall / n * 1e6:.1f}us")
    eng.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
