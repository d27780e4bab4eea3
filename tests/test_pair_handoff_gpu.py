"""Two data-parallel engines in ONE process on ONE GPU, joined by a device loopback
all-reduce (``parallel.comm.LoopbackPair``): each engine's comm work -- pre-issued
counter waits + collectives on its own high-priority comm stream, or collectives
captured in its step graph -- depends on the OTHER engine's compute replay, the
cross-rank dependency a 1-rank RCCL group never creates, under the box's
hardware-queue limit (GPU_MAX_HW_QUEUES, 4 by default; four streams here plus the
null stream).  The replicas must stay bit-identical and match one engine stepping
on the concatenated batch (multi_gpu_trainer.py:88,128: DDP's bucketed all-reduce
overlapped with backward).

Covered: the event-split pre-issued layout (overlap-2, comm stream ahead of the
compute replay) and the captured inline layout with 4-step graphs (graph-inline-1).
Not covered: the captured comm-BRANCH layout (graph-overlap-*, not an autotune
candidate): in one process its graph branches run on runtime-internal streams that
can share a hardware queue with the other engine's graph, and the loopback
all-reduce then waits out its bound (measured on MI355X, round 5) -- an artifact of
two ranks in one process that separate rank processes do not have.
"""
import pytest
import torch

from ddim_cold_amd import build_model
from ddim_cold_amd.parallel.comm import LoopbackPair
from ddim_cold_amd.train.engine import EngineConfig, TrainEngine

pytestmark = pytest.mark.gpu

B = 8  # per engine
LR = 1e-3
TIMEOUT_US = 500_000


def _batch(n):
    g = torch.Generator().manual_seed(11)
    x = torch.randn(n, 3, 64, 64, generator=g).clamp(-1, 1).cuda()
    y = torch.randn(n, 3, 64, 64, generator=g).clamp(-1, 1).cuda()
    t = torch.randint(1, 7, (n,), generator=g).cuda()
    return x, y, t


def _engine(dp: bool, K: int = 1):
    torch.manual_seed(100)
    model = build_model("vit_tiny", drop_rate=0.0, attn_drop_rate=0.0, drop_path_rate=0.0).cuda().train()
    cfg = EngineConfig(lr=LR, t_max=100, seed=5, temb_rows=7, graph_warmup=1, force_segments=dp, graph_steps=K)
    return TrainEngine(model, cfg)


@pytest.mark.parametrize("layout,K", [("overlap-2", 1), ("graph-inline-1", 4)])
def test_two_engines_cross_queue_handoff(layout, K, monkeypatch):
    monkeypatch.setenv("DDIM_COLD_HANDOFF_TIMEOUT_US", str(TIMEOUT_US))
    x, y, t = _batch(2 * B)
    engs = [_engine(True, K), _engine(True, K)]
    pair = LoopbackPair("cuda", engs[0].numel, timeout_us=TIMEOUT_US)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for e, eng in enumerate(engs):
        eng.attach_comm(pair.endpoint(e), 2)
        eng.apply_layout(layout)
        sl = slice(e * B, (e + 1) * B)
        st = (x[sl].clone(), y[sl].clone(), t[sl].clone())
        eng.set_batch_fn(lambda st=st: st)
    n_eager, n_graph = 1, 8
    for _ in range(n_eager):  # eager steps in lockstep
        for eng, s in zip(engs, streams):
            with torch.cuda.stream(s):
                eng.train_step()
    # capture BOTH before either replays: a capture synchronizes the device, which
    # would wait for the other engine's pre-issued collectives (one process, one GPU)
    for eng, s in zip(engs, streams):
        with torch.cuda.stream(s):
            eng._capture()
    done = 0
    while done < n_graph:
        for eng, s in zip(engs, streams):
            with torch.cuda.stream(s):
                eng.train_steps(K, materialize=False)
        done += K
    for eng, s in zip(engs, streams):
        with torch.cuda.stream(s):
            eng.materialize_lazy()
    torch.cuda.synchronize()
    assert not pair.failed(), f"loopback all-reduce wait timed out ({layout})"
    assert not any(eng.comm_error() for eng in engs), f"hand-off wait timed out ({layout})"
    if layout == "overlap-2":
        assert all(eng.handoff_order == "pre-issued" for eng in engs), [eng.handoff_order for eng in engs]
    else:
        assert all(len(eng._graphs) == 1 and eng._multi is not None for eng in engs)
    assert torch.equal(engs[0].flat_p, engs[1].flat_p), "replicas diverged"
    assert torch.equal(engs[0].flat_m, engs[1].flat_m)
    # one engine on the concatenated batch (the all-reduce SUM / 2 == the full-batch mean)
    ref = _engine(False)
    ref.set_batch_fn(lambda: (x, y, t))
    for _ in range(n_eager + n_graph):
        ref.train_step()
    torch.cuda.synchronize()
    dp = (engs[0].flat_p - ref.flat_p).abs().max().item()
    # AdamW turns last-bit gradient differences (batch split, bf16 rounding) into at most
    # ~2 lr per step; a collective that ran on stale or partial gradients moves whole
    # ranges by O(lr) every step in the same direction -- and breaks the loss
    assert dp <= 2 * LR * (n_eager + n_graph), (layout, dp)
    dl = abs(float(engs[0].loss_last) * 0.5 + float(engs[1].loss_last) * 0.5 - float(ref.loss_last))
    assert dl <= 1e-3 * abs(float(ref.loss_last)), (layout, dl)


def test_attach_comm_rejects_sparse_temb_engine_without_all_gather():
    """A Gaussian-diffusion engine (temb_rows None) exchanges the time-embedding
    gradient by all-gather; the loopback endpoint has only all_reduce_, so attaching it
    must fail up front instead of at the first step."""
    torch.manual_seed(100)
    model = build_model("vit_tiny").cuda().train()
    eng = TrainEngine(model, EngineConfig(lr=LR, t_max=100, seed=5, temb_rows=None, force_segments=True))
    pair = LoopbackPair("cuda", eng.numel)
    with pytest.raises(ValueError, match="all_gather_"):
        eng.attach_comm(pair.endpoint(0), 2)
