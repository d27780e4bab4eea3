"""Two ranks on ONE GPU: the data-parallel step with real cross-rank gradient traffic.

RCCL refuses two ranks on one device, so the process group here is gloo (CUDA
tensors, host-staged); everything else is the multi-GPU code path: rank-0
broadcast of the parameters, per-bucket ranges, the event-split step graphs
with host-issued collectives on the comm stream, autotune_comm() (timed layouts,
max over ranks, training state restored), and the optimizer on the summed
gradients.  Checked against one process stepping on the concatenated batch
(no dropout): losses, first Adam moments and parameters after 3 steps, and the
replicas bit-identical.

    python tools/dist2_gpu.py      (prints "dist2-gpu ok")
"""
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ddim_cold_amd.models import build_model
from ddim_cold_amd.train.engine import EngineConfig, TrainEngine

B = 16  # per rank
STEPS = 3


def _batches(n):
    g = torch.Generator().manual_seed(11)
    out = []
    for _ in range(STEPS):
        x = torch.randn(n, 3, 64, 64, generator=g).clamp(-1, 1)
        y = torch.randn(n, 3, 64, 64, generator=g).clamp(-1, 1)
        t = torch.randint(1, 7, (n,), generator=g)
        out.append((x, y, t))
    return out


def _engine(seed_model, world):
    torch.manual_seed(seed_model)
    model = build_model("vit_tiny", drop_rate=0.0, attn_drop_rate=0.0, drop_path_rate=0.0).cuda().train()
    cfg = EngineConfig(lr=1e-3, t_max=100, seed=5, temb_rows=7, graph_warmup=1)
    return TrainEngine(model, cfg)


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        eng = _engine(100 + rank, world)  # different init per rank: rank 0's is broadcast
        assert eng.segmented and eng.cfg.comm_events
        bs = [tuple(a[rank * B:(rank + 1) * B].cuda() for a in b) for b in _batches(world * B)]
        snap = eng._snapshot_state()
        eng.step(*bs[0])  # builds the static batch buffers the graphs read ...
        eng._restore_state(snap)  # ... and is undone
        times = eng.autotune_comm(steps=3, warm=1)
        # gloo cannot be captured: the captured (graph-) layouts are not candidates
        assert set(times) >= {L[0] for L in eng.COMM_LAYOUTS if not L[0].startswith("graph-")}, times
        losses = []
        for x, y, t in bs:
            eng.step(x, y, t)
            losses.append(float(eng.loss_last))
        torch.cuda.synchronize()
        p = eng.flat_p.clone()
        ps = [torch.empty_like(p) for _ in range(world)]
        dist.all_gather(ps, p)
        if rank == 0:
            torch.save({"p": p.cpu(), "m": eng.flat_m.cpu(), "losses": losses, "choice": eng.comm_choice,
                        "same": all(torch.equal(ps[0], q) for q in ps), "times": times}, out)
    finally:
        dist.destroy_process_group()



def main():
    from ddim_cold_amd.parallel.dist import free_port
    world = 2
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r.pt")
        mp.start_processes(_worker, args=(world, free_port(), out), nprocs=world, join=True, start_method="spawn")
        r = torch.load(out, weights_only=True)
    assert r["same"], "replicas diverged"
    # single process on the concatenated batches, from rank 0's init
    bs = [tuple(a.cuda() for a in b) for b in _batches(world * B)]
    eng2 = _engine(100, 1)
    losses = []
    for x, y, t in bs:
        eng2.step(x, y, t)
        losses.append(float(eng2.loss_last))
    torch.cuda.synchronize()
    # per-rank loss = mean over the rank's half; the single-process loss = mean over both halves
    print("losses 2-rank(rank0 half)", [round(v, 6) for v in r["losses"]], "single", [round(v, 6) for v in losses])
    dm = (r["m"] - eng2.flat_m.cpu()).abs().max().item() / eng2.flat_m.abs().max().item()
    dp = (r["p"] - eng2.flat_p.cpu()).abs().max().item()
    print(f"layout {r['choice']} times {r['times']}; rel |dm| {dm:.2e}; max |dp| {dp:.2e}")
    assert dm < 2e-2, dm
    assert dp <= 2 * 1e-3 * STEPS, dp
    print("dist2-gpu ok")


if __name__ == "__main__":
    main()
