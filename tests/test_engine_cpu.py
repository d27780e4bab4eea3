"""TrainEngine semantics on CPU: AdamW/clip/cosine vs torch.optim, optimizer-state formats,
and data-parallel gradient parity over gloo (world size 2)."""
import os
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ddim_cold_amd.models import DiffusionVisionTransformer
from ddim_cold_amd.models.program import collect, is_matrix_param
from ddim_cold_amd.ops import reference as ref
from ddim_cold_amd.parallel.dist import free_port
from ddim_cold_amd.train.engine import EngineConfig, TrainEngine

CFG = dict(img_size=[16, 16], patch_size=4, embed_dim=32, depth=3, num_heads=2)


def _model(drop=True, seed=0, **extra):
    torch.manual_seed(seed)
    kw = dict(drop_rate=0.1, attn_drop_rate=0.1, drop_path_rate=0.2) if drop else dict(drop_rate=0.0, attn_drop_rate=0.0, drop_path_rate=0.0)
    return DiffusionVisionTransformer(**CFG, **kw, **extra).train()


def _batch(B, seed=1):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, 3, 16, 16, generator=g)
    y = torch.randn(B, 3, 16, 16, generator=g).clamp(-1, 1)
    t = torch.randint(0, 2000, (B,), generator=g)
    return x, y, t


def _grads(model, x, y, t, rng):
    """Gradients of one step computed directly with the program (bf16 shadow weights, like the engine)."""
    from ddim_cold_amd.models.program import ViTProgram
    prog = ViTProgram.from_model(model)
    c = prog.cfg
    views = {n: (p.detach().to(torch.bfloat16) if is_matrix_param(n) else p.detach())
             for n, p in model.named_parameters()}
    grads = {n: torch.zeros_like(p) for n, p in model.named_parameters()}
    P = collect(views, c.depth, c.dim)
    from ddim_cold_amd.models import program as pr
    if pr.FOLD_LN:  # the engine folds every LayerNorm into its consumer GEMM
        fold = pr.LnFold({n: p.detach() for n, p in model.named_parameters()}, c.depth,
                         weights={n: v for n, v in views.items() if is_matrix_param(n)})
        fold.refresh()
        fold.attach(P)
    G = collect(grads, c.depth, c.dim)
    out, S = prog.forward(P, x, t, rng, True)
    loss, dtok = ref.smooth_l1_fwd_bwd(out, y, c.tokens, c.patch)
    prog.backward(P, G, S, dtok, rng, True)
    return grads, float(loss)


def test_engine_matches_torch_adamw_clip_cosine():
    model = _model()
    ref_model = _model()
    cfg = EngineConfig(lr=1e-3, t_max=5, max_grad_norm=0.05, seed=11)
    eng = TrainEngine(model, cfg, device="cpu")
    opt = torch.optim.AdamW(ref_model.parameters(), lr=1e-3, betas=cfg.betas, eps=cfg.eps, weight_decay=0.05)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, 5)
    names = [n for n, _ in ref_model.named_parameters()]
    for step in range(3):
        x, y, t = _batch(4, seed=step)
        g, loss_val = _grads(ref_model, x, y, t, torch.tensor([11, step]))
        for n, p in ref_model.named_parameters():
            p.grad = g[n].clone()
        torch.nn.utils.clip_grad_norm_(ref_model.parameters(), 0.05)
        opt.step()
        sched.step()
        loss = eng.step(x, y, t)
        assert float(loss) == pytest.approx(loss_val, rel=1e-6)
    sd_e, sd_r = model.state_dict(), ref_model.state_dict()
    for n in names:
        assert torch.allclose(sd_e[n], sd_r[n], atol=2e-6, rtol=1e-5), n
    assert eng.current_lr() == pytest.approx(sched.get_last_lr()[0])
    assert int(eng.step_ctr[0]) == 3 and int(eng.rng[1]) == 3
    # optimizer / scheduler state dicts load into the torch classes (reference lastepoch.pkl layout)
    osd = eng.optimizer_state_dict()
    o2 = torch.optim.AdamW(_model().parameters(), lr=1e-3, weight_decay=0.05)
    o2.load_state_dict(osd)
    st_r = opt.state_dict()["state"]
    for i in range(len(names)):
        assert torch.allclose(osd["state"][i]["exp_avg"], st_r[i]["exp_avg"], atol=1e-7)
        assert float(osd["state"][i]["step"]) == 3
    ssd = eng.scheduler_state_dict()
    s2 = torch.optim.lr_scheduler.CosineAnnealingLR(o2, 5)
    s2.load_state_dict(ssd)
    assert s2.last_epoch == 3
    # round trip into a fresh engine
    eng2 = TrainEngine(_model(), cfg, device="cpu")
    eng2.load_optimizer_state_dict(osd)
    eng2.load_scheduler_state_dict(ssd)
    assert torch.equal(eng2.flat_m, eng.flat_m) and torch.equal(eng2.flat_v, eng.flat_v)
    assert int(eng2.step_ctr[0]) == 3 and int(eng2.step_ctr[1]) == 3


def test_engine_frozen_sinusoidal_table_matches_torch_adamw():
    """A requires_grad=False parameter (the fixed sinusoidal timestep table,
    ViT_draft2drawing.py:140-156) is left alone by the fused optimizer exactly as
    torch.optim.AdamW leaves a parameter whose .grad is None: no weight decay, no
    moments, no state entry; every other parameter matches torch step for step."""
    from ddim_cold_amd.models.vit import positionalencoding1d
    model = _model(timestep_embedding="sinusoidal")
    ref_model = _model(timestep_embedding="sinusoidal")
    table0 = positionalencoding1d(CFG["embed_dim"], 2000)
    assert torch.equal(model.time_embed.weight.detach(), table0)
    cfg = EngineConfig(lr=1e-3, t_max=20, max_grad_norm=0.05, seed=11)  # decay would move every element
    eng = TrainEngine(model, cfg, device="cpu")
    assert "time_embed.weight" in eng.frozen and eng.offsets["time_embed.weight"][0] >= eng.train_hi
    assert model.time_embed.weight.grad is None
    assert all(b <= eng.train_hi for _, b in eng.buckets)
    opt = torch.optim.AdamW(ref_model.parameters(), lr=1e-3, betas=cfg.betas, eps=cfg.eps, weight_decay=0.05)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, 20)
    for step in range(3):
        x, y, t = _batch(4, seed=step)
        g, loss_val = _grads(ref_model, x, y, t, torch.tensor([11, step]))
        for n, p in ref_model.named_parameters():
            p.grad = g[n].clone() if p.requires_grad else None
        torch.nn.utils.clip_grad_norm_([p for p in ref_model.parameters() if p.requires_grad], 0.05)
        opt.step()
        sched.step()
        loss = eng.step(x, y, t)
        assert float(loss) == pytest.approx(loss_val, rel=1e-6)
    sd_e, sd_r = model.state_dict(), ref_model.state_dict()
    for n in sd_r:
        assert torch.allclose(sd_e[n], sd_r[n], atol=2e-6, rtol=1e-5), n
    for step in range(3, 10):  # 10 steps in all
        eng.step(*_batch(4, seed=step))
    assert torch.equal(model.time_embed.weight.detach(), table0)  # bit-identical after training
    names = [n for n, _ in model.named_parameters()]
    osd = eng.optimizer_state_dict()
    assert names.index("time_embed.weight") not in osd["state"]
    assert len(osd["state"]) == len(names) - 1
    o2 = torch.optim.AdamW(_model(timestep_embedding="sinusoidal").parameters(), lr=1e-2, weight_decay=0.05)
    o2.load_state_dict(osd)


def test_engine_params_are_arena_views():
    model = _model()
    eng = TrainEngine(model, EngineConfig(), device="cpu")
    for n, p in model.named_parameters():
        o, k = eng.offsets[n]
        assert p.data.data_ptr() == eng.flat_p[o:].data_ptr()
        assert p.grad.data_ptr() == eng.flat_g[o:].data_ptr()
        is_ln_bias = n.endswith(".bias") and p.dim() == 1 and "norm" in n
        assert o % 64 == 0 or (is_ln_bias and o % 4 == 0), n
    # buckets tile the arena exactly
    cover = sorted(eng.buckets)
    assert cover[0][0] == 0 and cover[-1][1] == eng.numel
    assert all(a[1] == b[0] for a, b in zip(cover, cover[1:]))


def test_nonfinite_grad_skips_update():
    model = _model()
    eng = TrainEngine(model, EngineConfig(), device="cpu")
    before = eng.flat_p.clone()
    x, y, t = _batch(2)
    x[0, 0, 0, 0] = float("nan")
    eng.step(x, y, t)
    assert torch.equal(eng.flat_p, before)
    assert int(eng.step_ctr[0]) == 0 and int(eng.step_ctr[1]) == 1


def _ddp_worker(rank, world, port, out_path, wire="fp32", gauss=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        model = _model(drop=False, seed=rank)  # different init per rank: engine must broadcast rank 0's
        eng = TrainEngine(model, EngineConfig(lr=1e-3, weight_decay=0.0, max_grad_norm=0.0, bucket_blocks=1,
                                              temb_rows=None if gauss else 7, grad_wire=wire), device="cpu")
        # inactive time_embed rows skipped (cold) or the whole table exchanged as
        # all-gathered rows (Gaussian); the embeddings have their own last bucket
        reduced = sum(b - a for rs in eng.bucket_ranges for a, b in rs)
        assert reduced == eng.numel - (2000 - (0 if gauss else 7)) * model.embed_dim
        assert (eng.temb_bucket is not None) == gauss
        assert eng.bucket_ranges[-1][-1][1] <= eng.offsets["blocks.0.attn.qkv.weight"][0]
        # every LayerNorm sits in the last (embedding) bucket: finalised once, after block 0
        last = eng.buckets[-1]
        assert all(last[0] <= eng.offsets[n][0] < last[1] for n in eng.names if ".norm" in n or n.startswith("norm"))
        x, y, t = _batch(4, seed=5)
        t = t % 6 + 1 if not gauss else t[[0, 0, 1, 0]]  # cold timesteps / repeats across and within ranks
        b = 4 // world
        eng.step(x[rank * b:(rank + 1) * b], y[rank * b:(rank + 1) * b], t[rank * b:(rank + 1) * b])
        m = eng.flat_m.clone()
        ms = [torch.zeros_like(m) for _ in range(world)]
        dist.all_gather(ms, m)
        if rank == 0:
            torch.save({"m": m, "p": eng.flat_p.clone(), "same": all(torch.equal(ms[0], q) for q in ms)},
                       out_path)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("wire,tol,gauss", [("fp32", 1e-4, False), ("bf16", 2e-2, False), ("fp32", 1e-4, True)])
def test_data_parallel_gloo_matches_single_process(wire, tol, gauss):
    """Bucketed all-reduce over 2 ranks == one process on the full batch (no dropout);
    gauss: sparse time_embed row exchange, with a t repeated inside and across ranks."""
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r.pt")
        mp.start_processes(_ddp_worker, args=(2, free_port(), out, wire, gauss), nprocs=2, join=True,
                           start_method="spawn")
        r = torch.load(out, weights_only=True)
    assert r["same"]
    model = _model(drop=False, seed=0)
    eng = TrainEngine(model, EngineConfig(lr=1e-3, weight_decay=0.0, max_grad_norm=0.0), device="cpu")
    x, y, t = _batch(4, seed=5)
    eng.step(x, y, t[[0, 0, 1, 0]] if gauss else t % 6 + 1)
    m1 = eng.flat_m
    # exp_avg after one step = (1-b1) * mean-gradient
    err = (r["m"] - m1).abs().max().item() / m1.abs().max().item()
    assert err < tol, err
    o, k = eng.offsets["time_embed.weight"]
    te, te1 = r["m"][o:o + k], m1[o:o + k]
    assert te1.abs().max() > 0 and (te - te1).abs().max().item() < tol * te1.abs().max().item()


def test_grad_accumulation_matches_full_batch():
    """grad_accum=2 over two half batches == one step on the full batch (no dropout)."""
    x, y, t = _batch(4, seed=9)
    full = TrainEngine(_model(drop=False), EngineConfig(lr=1e-3, weight_decay=0.0, max_grad_norm=0.0), device="cpu")
    full.step(x, y, t)
    acc = TrainEngine(_model(drop=False), EngineConfig(lr=1e-3, weight_decay=0.0, max_grad_norm=0.0, grad_accum=2),
                      device="cpu")
    halves = iter([(x[:2], y[:2], t[:2]), (x[2:], y[2:], t[2:])])
    acc.set_batch_fn(lambda: next(halves))
    acc.train_step()
    err = (acc.flat_m - full.flat_m).abs().max().item() / full.flat_m.abs().max().item()
    assert err < 1e-4, err
    assert int(acc.step_ctr[0]) == 1 and int(acc.rng[1]) == 2
    # one EMA update per optimizer step with the mean micro-batch loss
    # (multi_gpu_trainer.py:126: loss_rec = 0.99 loss_rec + 0.01 loss)
    torch.testing.assert_close(acc.loss_last, full.loss_last, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(acc.loss_ema, 0.99 * 5.0 + 0.01 * full.loss_last, rtol=1e-5, atol=1e-6)


def test_grad_accumulation_ema_once_per_step_without_fold(monkeypatch):
    """Same EMA semantics on the unfolded path (no step tail)."""
    x, y, t = _batch(4, seed=9)
    acc = TrainEngine(_model(drop=False), EngineConfig(lr=1e-3, weight_decay=0.0, max_grad_norm=0.0, grad_accum=2),
                      device="cpu")
    acc.lnfold = None
    halves = iter([(x[:2], y[:2], t[:2]), (x[2:], y[2:], t[2:])])
    acc.set_batch_fn(lambda: next(halves))
    acc.train_step()
    assert int(acc.step_ctr[0]) == 1 and int(acc.rng[1]) == 2
    torch.testing.assert_close(acc.loss_ema, 0.99 * 5.0 + 0.01 * acc.loss_last, rtol=1e-5, atol=1e-6)


def _sync_worker(rank, world, port, out_path):
    from ddim_cold_amd.utils.observe import check_param_sync
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        same = torch.arange(10.0)
        check_param_sync(same)  # identical: passes
        try:
            check_param_sync(same + rank)  # diverged replicas
            ok = False
        except RuntimeError:
            ok = True
        if rank == 0:
            torch.save({"detected": ok}, out_path)
    finally:
        dist.destroy_process_group()


def test_param_sync_check_detects_divergence():
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r.pt")
        mp.start_processes(_sync_worker, args=(2, free_port(), out), nprocs=2, join=True, start_method="spawn")
        assert torch.load(out, weights_only=True)["detected"]


def test_reference_ksplit_dgrad_and_ln_partials():
    """K-split dgrad partials (64-aligned slices of the reduction dim) sum to the
    full product, and the LayerNorm backward accepts the stacked partials."""
    from ddim_cold_amd.ops import reference as ref
    torch.manual_seed(0)
    dy = torch.randn(40, 200).to(torch.bfloat16)
    w = torch.randn(200, 128).to(torch.bfloat16)
    parts = ref.linear_dgrad(dy, w, True, 3)
    assert parts.shape == (3, 40, 128)
    torch.testing.assert_close(parts.sum(0), ref.linear_dgrad(dy, w, True), rtol=1e-5, atol=1e-4)
    x = torch.randn(40, 128)
    g, b = torch.randn(128), torch.randn(128)
    _, mu, rs = ref.layernorm_fwd(x, g, b)
    r = torch.tensor([1, 2], dtype=torch.int64)
    z = [torch.zeros(128) for _ in range(4)]
    a, _ = ref.layernorm_bwd(parts, x, mu, rs, g, None, z[0], z[1], 40, r, 0, 0.0, 0, 0.0, False)
    e, _ = ref.layernorm_bwd(parts.sum(0), x, mu, rs, g, None, z[2], z[3], 40, r, 0, 0.0, 0, 0.0, False)
    torch.testing.assert_close(a, e)
    torch.testing.assert_close(z[0], z[2])


def test_engine_fused_cold_batch_matches_unfused_cpu():
    """ColdBatcher.fused_spec path (draw fused into the patch embedding) == the plain batch_fn path."""
    from ddim_cold_amd.data.synthetic import ColdBatcher, synthetic_pool

    def run(fuse):
        model = _model()
        eng = TrainEngine(model, EngineConfig(lr=1e-3, t_max=10, use_graph=False, seed=5, fuse_batch=fuse))
        bat = ColdBatcher(synthetic_pool(16, size=(16, 16), seed=1), 4, eng.rng)
        calls = []
        if fuse:
            spec = bat.fused_spec
            bat.fused_spec = lambda: (calls.append(1), spec())[1]
        eng.set_batch_fn(bat)
        losses = [float(eng.train_step()) for _ in range(3)]
        return eng.flat_p.clone(), losses, len(calls), bat.t.clone(), bat.x_tm1.clone()
    pf, lf, nf, tf, yf = run(True)
    pu, lu, _, tu, yu = run(False)
    from ddim_cold_amd import ops
    from ddim_cold_amd.models import program
    if program.TARGET_ROWS:  # the fused draw wrote the loss target as patch rows
        yf = ops.rows_to_image(yf.reshape(-1, 3 * 4 * 4), *yf.shape, 4)
    assert nf == 3  # the fused path really ran
    assert lf == lu and torch.equal(pf, pu) and torch.equal(tf, tu) and torch.equal(yf, yu)


def _layout_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        eng = TrainEngine(_model(drop=False, seed=rank), EngineConfig(lr=1e-3, temb_rows=7), device="cpu")
        x, y, t = _batch(4, seed=5)
        t = t % 6 + 1
        b = 4 // world
        xb, yb, tb = x[rank * b:(rank + 1) * b], y[rank * b:(rank + 1) * b], t[rank * b:(rank + 1) * b]
        snap = eng._snapshot_state()
        res = {}
        # the fixed layouts + model-picked bucket sizes (cost model candidates)
        lays = list(eng.COMM_LAYOUTS) + [eng.layout_by_name(n) for n in ("overlap-1", "overlap-3", "overlap-7")]
        for L in lays:
            name = L[0]
            eng.apply_layout(L)
            assert eng.comm_choice == name and eng.cfg.comm_events == (not name.startswith("graph-"))
            cover = sorted(eng.buckets)  # buckets tile the arena for every layout
            assert cover[0][0] == 0 and cover[-1][1] == eng.numel
            assert all(a[1] == c[0] for a, c in zip(cover, cover[1:]))
            if name.endswith("inline-1"):
                assert len(eng.buckets) == 1 and eng.comm is None
            eng.step(xb, yb, tb)
            eng.step(xb, yb, tb)
            res[name] = (eng.flat_p.clone(), eng.flat_m.clone(), eng.loss_ema.clone())
            eng._restore_state(snap)
        assert eng.autotune_comm() == {}  # CPU: nothing to tune
        if rank == 0:
            torch.save({k: list(v) for k, v in res.items()} | {"p0": snap[0]["flat_p"], "p_end": eng.flat_p.clone()},
                       out_path)
    finally:
        dist.destroy_process_group()


def test_comm_layouts_same_training_gloo():
    """Every gradient-exchange layout autotune_comm() chooses from (2- / 4-block buckets
    overlapped, one inline bucket) gives the same two training steps over 2 gloo ranks,
    and the snapshot / restore around the tuning steps leaves the state untouched."""
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r.pt")
        mp.start_processes(_layout_worker, args=(2, free_port(), out), nprocs=2, join=True, start_method="spawn")
        r = torch.load(out, weights_only=True)
    assert torch.equal(r["p0"], r["p_end"])
    base = r["overlap-2"]
    assert not torch.equal(base[0], r["p0"])
    for name in ("overlap-4", "inline-1", "graph-inline-1", "overlap-1", "overlap-3", "overlap-7"):
        for a, b in zip(base, r[name]):
            assert torch.equal(a, b), name


def test_lazy_time_embed_decay_matches_torch_adamw():
    """Cold training (t in 1..6, temb_rows=7): the optimizer skips the 1,993 time_embed
    rows no sample can select and accumulates their weight decay on the device;
    materialised, every parameter -- those rows included -- equals torch.optim.AdamW
    + clip + cosine on the same gradients (rows with zero gradient and moments
    decay as p *= 1 - lr*wd)."""
    model = _model()
    ref_model = _model()
    cfg = EngineConfig(lr=1e-3, t_max=5, max_grad_norm=0.05, seed=11, temb_rows=7)
    eng = TrainEngine(model, cfg, device="cpu")
    assert eng.lazy is not None
    lo, hi = eng.lazy
    o, k = eng.offsets["time_embed.weight"]
    assert lo == o + 7 * model.embed_dim and hi == o + k
    opt = torch.optim.AdamW(ref_model.parameters(), lr=1e-3, betas=cfg.betas, eps=cfg.eps, weight_decay=0.05)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, 5)
    before = eng.flat_p[lo:hi].clone()
    decay = 1.0
    batches = [_batch(4, seed=step) for step in range(3)]
    eng.set_batch_fn(iter([(x, y, t % 6 + 1) for x, y, t in batches]).__next__)
    for step, (x, y, t) in enumerate(batches):
        t = t % 6 + 1
        g, _ = _grads(ref_model, x, y, t, torch.tensor([11, step]))
        for n, p in ref_model.named_parameters():
            p.grad = g[n].clone()
        torch.nn.utils.clip_grad_norm_(ref_model.parameters(), 0.05)
        decay *= 1 - sched.get_last_lr()[0] * 0.05
        opt.step()
        sched.step()
        eng.train_step(materialize=False)
        assert torch.equal(eng.flat_p[lo:hi], before)  # untouched while training
        assert float(eng.lazy_decay) == pytest.approx(decay, rel=1e-6)
    eng.materialize_lazy()
    assert float(eng.lazy_decay) == 1.0 and not eng._lazy_dirty
    sd_e, sd_r = model.state_dict(), ref_model.state_dict()
    for n in sd_r:
        assert torch.allclose(sd_e[n], sd_r[n], atol=2e-6, rtol=1e-5), n
    assert torch.allclose(eng.flat_pb[lo:hi].float(), eng.flat_p[lo:hi].bfloat16().float())
    # moments of the lazy rows stay exactly zero; the state dict matches torch's
    osd = eng.optimizer_state_dict()
    i_t = [n for n, _ in ref_model.named_parameters()].index("time_embed.weight")
    assert torch.allclose(osd["state"][i_t]["exp_avg"], opt.state_dict()["state"][i_t]["exp_avg"], atol=1e-7)
    assert float(osd["state"][i_t]["exp_avg"][7:].abs().max()) == 0.0


def test_lazy_decay_snapshot_restore_and_load():
    """A snapshot (autotune_comm / checkpoints) is taken materialised; loading weights
    discards any pending decay."""
    model = _model()
    eng = TrainEngine(model, EngineConfig(lr=1e-3, t_max=50, seed=3, temb_rows=7), device="cpu")
    x, y, t = _batch(4, seed=1)
    eng.set_batch_fn(lambda: (x, y, t % 6 + 1))
    eng.train_steps(2, materialize=False)
    assert eng._lazy_dirty and float(eng.lazy_decay) < 1.0
    snap = eng._snapshot_state()
    assert not eng._lazy_dirty and float(eng.lazy_decay) == 1.0
    p_mat = eng.flat_p.clone()
    eng.train_steps(2, materialize=False)
    eng._restore_state(snap)
    assert torch.equal(eng.flat_p, p_mat) and float(eng.lazy_decay) == 1.0 and not eng._lazy_dirty
    eng.train_steps(1, materialize=False)
    eng.sync_params_from_model()
    assert float(eng.lazy_decay) == 1.0 and not eng._lazy_dirty


def test_resume_with_moments_on_lazy_rows_turns_lazy_off():
    """An optimizer state whose Adam moments are non-zero on the rows the cold run can
    never select (e.g. from a Gaussian-diffusion run) disables the lazy shortcut, so
    those rows keep their torch.optim.AdamW updates."""
    model = _model()
    eng = TrainEngine(model, EngineConfig(lr=1e-3, t_max=50, seed=3, temb_rows=7), device="cpu")
    assert eng.lazy is not None
    sd = eng._optimizer_sd(eng.flat_m, eng.flat_v, 0, 0)
    names = [n for n, _ in model.named_parameters()]
    i_t = names.index("time_embed.weight")
    shape = model.time_embed.weight.shape
    m = torch.zeros(shape)
    m[100] = 0.5
    sd["state"] = {i_t: {"step": torch.tensor(3.0), "exp_avg": m, "exp_avg_sq": m.abs()}}
    with pytest.warns(UserWarning, match="lazy weight decay off"):
        eng.load_optimizer_state_dict(sd)
    assert eng.lazy is None
    # zero moments there (a cold run's own checkpoint): the shortcut stays on
    eng2 = TrainEngine(_model(), EngineConfig(lr=1e-3, t_max=50, seed=3, temb_rows=7), device="cpu")
    sd["state"][i_t]["exp_avg"] = torch.zeros(shape)
    sd["state"][i_t]["exp_avg_sq"] = torch.zeros(shape)
    eng2.load_optimizer_state_dict(sd)
    assert eng2.lazy is not None
