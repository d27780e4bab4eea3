"""TrainEngine on the GPU: graph-captured steps (incl. gradient accumulation) agree with the
eager replay of the same step program."""
import pytest
import torch

from ddim_cold_amd import build_model
from ddim_cold_amd.data.synthetic import ColdBatcher, synthetic_pool
from ddim_cold_amd.train.engine import EngineConfig, TrainEngine


def _run(use_graph, grad_accum, steps=5):
    torch.manual_seed(0)
    model = build_model("vit_tiny").cuda().train()
    eng = TrainEngine(model, EngineConfig(lr=1e-3, t_max=100, seed=3, use_graph=use_graph, graph_warmup=1,
                                          grad_accum=grad_accum, temb_rows=7))
    eng.set_batch_fn(ColdBatcher(synthetic_pool(64, seed=1, device="cuda"), 8, eng.rng))
    losses = []
    for _ in range(steps):
        losses.append(float(eng.train_step()))
    torch.cuda.synchronize()
    return eng.flat_p.clone(), losses, eng


@pytest.mark.gpu
@pytest.mark.parametrize("grad_accum", [1, 2])
def test_graph_step_matches_eager(grad_accum):
    pg, lg, eng = _run(True, grad_accum)
    pe, le, _ = _run(False, grad_accum)
    assert eng._graphs is not None and len(eng._graphs) == 1
    # the graph replays exactly the eager step's kernels; no fp32 atomics: bit-identical
    assert lg == le, (lg, le)
    assert torch.equal(pg, pe)
    assert int(eng.rng[1]) == 5 * grad_accum and int(eng.step_ctr[0]) == 5


@pytest.mark.gpu
@pytest.mark.parametrize("target", ["prev", "x0"])
@pytest.mark.parametrize("draw", [True, False])
@pytest.mark.parametrize("name", ["vit_tiny", "oxford_flower"])  # patch 8 / patch 4 segments
def test_patch_embed_cold_matches_cold_batch_then_embed(target, draw, name):
    """ops.patch_embed_cold_fwd (batch draw fused into the patchify launch) == cold_batch
    followed by patch_embed_fwd, bit for bit (tokens, patch rows, target, t, idx, LN stats)."""
    from ddim_cold_amd import ops
    from ddim_cold_amd.data.synthetic import SITE_DATA
    from ddim_cold_amd.models.program import SITE_EMBED
    torch.manual_seed(0)
    model = build_model(name).cuda().train()
    B, D = 8, model.embed_dim
    N = model.patch_embed.num_patches + 1
    pool = synthetic_pool(32, seed=2, device="cuda")
    rng = torch.tensor([11, 5], dtype=torch.int64, device="cuda")
    idx0 = torch.randint(0, 32, (B,), device="cuda")
    pe_w = model.patch_embed.proj.weight.detach().reshape(D, -1).to(torch.bfloat16).contiguous()
    args = (pe_w, model.patch_embed.proj.bias.detach(), model.cls_token.detach(), model.pos_embed.detach(),
            model.time_embed.weight.detach(), rng, SITE_EMBED, 0.1, model.patch_size)

    def bufs():
        return (torch.empty(B, 3, 64, 64, device="cuda"), torch.empty(B, 3, 64, 64, device="cuda"),
                torch.empty(B, dtype=torch.int64, device="cuda"), idx0.clone(),
                torch.empty(B * N, D // 32, 2, device="cuda"), torch.empty(B * N, D, dtype=torch.bfloat16, device="cuda"))

    xt, tg, t, idx, st, xb = bufs()
    ops.cold_batch(pool, rng, SITE_DATA, xt, tg, t, idx, 6, draw)
    if target == "x0":
        torch.index_select(pool, 0, idx, out=tg)
    x_ref, p_ref = ops.patch_embed_fwd(xt, t, *args, ln_st=st, xb_out=xb)
    xt2, tg2, t2, idx2, st2, xb2 = bufs()
    cold = (pool, SITE_DATA, 6, draw, target == "x0", tg2, idx2, True)
    x, p = ops.patch_embed_cold_fwd(cold, xt2, t2, *args, ln_st=st2, xb_out=xb2)
    torch.cuda.synchronize()
    assert torch.equal(t2, t) and torch.equal(idx2, idx)
    assert torch.equal(xt2, xt) and torch.equal(tg2, tg)
    assert torch.equal(p, p_ref) and torch.equal(x, x_ref) and torch.equal(xb2, xb) and torch.equal(st2, st)


@pytest.mark.gpu
def test_engine_fused_batch_matches_unfused():
    def run(fuse):
        torch.manual_seed(0)
        model = build_model("vit_tiny").cuda().train()
        eng = TrainEngine(model, EngineConfig(lr=1e-3, t_max=100, seed=3, use_graph=True, graph_warmup=1,
                                              temb_rows=7, fuse_batch=fuse))
        eng.set_batch_fn(ColdBatcher(synthetic_pool(64, seed=1, device="cuda"), 8, eng.rng))
        losses = [float(eng.train_step()) for _ in range(4)]
        torch.cuda.synchronize()
        return eng.flat_p.clone(), losses
    pf, lf = run(True)
    pu, lu = run(False)
    pf2, lf2 = run(True)
    # no gradient reduction uses fp32 atomics (LayerNorm dgamma/dbeta: ordered in-launch
    # group sums; time embedding: one writer per row): two identical runs are
    # bit-identical after 4 steps
    assert lf == lf2, (lf, lf2)
    assert torch.equal(pf, pf2)
    # fused vs unfused draw bit-identical batches (test above) but sum the loss in a
    # different order (target as patch rows in the vector loss epilogue): last-bit
    # differences of the loss scale that AdamW turns into <= ~2 lr per step
    assert all(abs(a - b) <= 2e-4 * abs(b) for a, b in zip(lf, lu)), (lf, lu)
    assert (pf - pu).abs().max().item() <= 2 * 1e-3 * 4


@pytest.mark.gpu
def test_multi_step_graph_matches_single_step_graph():
    """train_steps with a 4-step graph == 9 single-step replays (every counter on the device)."""
    def run(K):
        torch.manual_seed(0)
        model = build_model("vit_tiny").cuda().train()
        eng = TrainEngine(model, EngineConfig(lr=1e-3, t_max=100, seed=3, use_graph=True, graph_warmup=1,
                                              temb_rows=7, graph_steps=K))
        eng.set_batch_fn(ColdBatcher(synthetic_pool(64, seed=1, device="cuda"), 8, eng.rng))
        eng.train_steps(9)  # 1 eager + capture, then (K=4) two 4-step replays
        torch.cuda.synchronize()
        return eng.flat_p.clone(), float(eng.loss_ema), eng
    pm, em, eng = run(4)
    ps, es, _ = run(1)
    assert eng._multi is not None and eng._multi[1] == 4 and eng.steps_done == 9
    assert int(eng.step_ctr[0]) == 9 and int(eng.rng[1]) == 9
    assert abs(em - es) <= 1e-4 * abs(es), (em, es)
    assert (pm - ps).abs().max().item() <= 2 * 1e-3 * 9


@pytest.mark.gpu
@pytest.mark.parametrize("graph", [False, True])
def test_fused_grad_norm_matches_sqnorm_pass(monkeypatch, graph):
    """Grad-norm partials written by the weight-gradient launch (engine.FUSE_SQNORM,
    default) == the separate sqnorm pass: same squared norm of the step's gradient
    (clipping active: a norm error would move every parameter), same parameters and
    counters after several steps (lazy time-embedding range on)."""
    from ddim_cold_amd.train import engine as engine_mod

    def run(flag):
        monkeypatch.setattr(engine_mod, "FUSE_SQNORM", flag)
        torch.manual_seed(0)
        model = build_model("vit_tiny").cuda().train()
        eng = TrainEngine(model, EngineConfig(lr=1e-3, t_max=100, seed=3, use_graph=graph, graph_warmup=1,
                                              temb_rows=7, max_grad_norm=0.1))
        eng.set_batch_fn(ColdBatcher(synthetic_pool(64, seed=1, device="cuda"), 8, eng.rng))
        eng.train_step()
        torch.cuda.synchronize()
        sq1 = eng.sqnorm.double().sum().item()
        eng.train_steps(5)
        torch.cuda.synchronize()
        return sq1, eng.flat_p.clone(), eng.step_ctr.clone(), float(eng.loss_ema)
    sf, pf, cf, ef = run(True)
    su, pu, cu, eu = run(False)
    assert sf > 0.01, "clipping (max norm 0.1) must be active for the comparison to mean anything"
    assert abs(sf - su) <= 1e-5 * su, (sf, su)
    assert torch.equal(cf, cu)
    assert abs(ef - eu) <= 1e-5 * abs(eu)
    # AdamW turns last-bit differences of near-zero grads (fp32 atomics) into <= 2*lr per step
    assert (pf - pu).abs().max().item() <= 2 * 1e-3 * 6


@pytest.mark.gpu
def test_ln_replica_finalize_fused_matches_separate(monkeypatch):
    """LayerNorm dgamma/dbeta replica finalize carried by the embedding-backward launch
    (engine.FUSE_LN_FINAL, default) == the separate replica_reduce_ launch:
    same LayerNorm parameters after the step (bit-identical: both sum the workspace
    slots in order)."""
    from ddim_cold_amd.train import engine as engine_mod

    def run(flag):
        monkeypatch.setattr(engine_mod, "FUSE_LN_FINAL", flag == "1")
        torch.manual_seed(0)
        model = build_model("vit_tiny").cuda().train()
        # no clipping: LayerNorm params after one AdamW step depend only on their own grads
        eng = TrainEngine(model, EngineConfig(lr=1e-3, t_max=100, seed=3, use_graph=False, temb_rows=7,
                                              max_grad_norm=0.0))
        eng.set_batch_fn(ColdBatcher(synthetic_pool(64, seed=1, device="cuda"), 8, eng.rng))
        eng.train_step()
        torch.cuda.synchronize()
        ln = torch.cat([eng.flat_p[eng.offsets[n + ".weight"][0]:eng.offsets[n + ".weight"][0] + 2 * model.embed_dim]
                        for n in eng.ln_order])
        # the step must have touched every LayerNorm parameter
        return ln.clone(), eng.flat_m.clone()
    lf, mf = run("1")
    lu, mu = run("0")
    init = torch.cat([torch.ones(384), torch.zeros(384)]).cuda().repeat(15)
    assert (lf - init).abs().max() > 0
    assert torch.equal(lf, lu)


@pytest.mark.gpu
def test_gradient_overwrite_matches_accumulate(monkeypatch):
    """Single writer per gradient range (tail weight-gradient launch and LayerNorm finalize
    store, AdamW zeroes only the embeddings) == accumulate + zero everything."""
    orig = TrainEngine._grad_overwrite

    def run(flag):
        monkeypatch.setattr(TrainEngine, "_grad_overwrite",
                            orig if flag == "1" else (lambda self, *a, **k: False))
        torch.manual_seed(0)
        model = build_model("vit_tiny").cuda().train()
        eng = TrainEngine(model, EngineConfig(lr=1e-3, t_max=100, seed=3, use_graph=True, graph_warmup=1,
                                              temb_rows=7))
        eng.set_batch_fn(ColdBatcher(synthetic_pool(64, seed=1, device="cuda"), 8, eng.rng))
        losses = [float(eng.train_step()) for _ in range(5)]
        torch.cuda.synchronize()
        return eng.flat_p.clone(), losses, eng
    po, lo, eng = run("1")
    pa, la, eng_a = run("0")
    assert eng.acc_hi < eng.offsets["blocks.0.attn.qkv.weight"][0]
    # overwrite mode leaves the last step's gradients above acc_hi in place; accumulate zeroes all
    assert eng.flat_g[eng.acc_hi:].abs().max() > 0 and eng_a.flat_g.abs().max() == 0
    assert eng.flat_g[:eng.acc_hi].abs().max() == 0
    assert all(abs(a - b) <= 1e-4 * abs(b) for a, b in zip(lo, la)), (lo, la)
    assert (po - pa).abs().max().item() <= 2 * 1e-3 * 5


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["cold", "gaussian"])
def test_graph_evaluate_matches_eager(kind):
    """trainer.evaluate: full validation batches replayed from a captured graph (index buffer,
    batch draw, forward, device loss sum) == the eager loop; ragged tail batch eager."""
    from ddim_cold_amd.train.trainer import evaluate
    torch.manual_seed(0)
    model = build_model("vit_tiny").cuda().train()
    pool = synthetic_pool(40, seed=4, device="cuda")
    idx = torch.randperm(40)[:37]
    vals = []
    for use_graph in (True, False):
        eng = TrainEngine(model, EngineConfig(use_graph=use_graph, temb_rows=7))
        rng = torch.tensor([123, 0], dtype=torch.int64, device="cuda")
        v1 = evaluate(model, eng, pool, idx, 8, kind, 2000, rng)
        v2 = evaluate(model, eng, pool, idx, 8, kind, 2000, rng)  # second call replays the cached graph
        assert int(rng[1]) == 2 * 5
        vals.append((v1, v2))
        eng.detach()
    (g1, g2), (e1, e2) = vals
    assert abs(g1 - e1) <= 1e-6 * abs(e1) and abs(g2 - e2) <= 1e-6 * abs(e2), vals


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["cold", "gaussian"])
def test_grouped_graph_evaluate(kind, monkeypatch):
    """EVAL_GROUP full batches per replay (one forward of 8 x batch images): the same
    estimator as one batch per replay -- equal batch sizes, so the mean of batch means
    is the mean over the group (the batch draws differ: compared over 1,000 samples) --
    with the leftover full batches (3) and the ragged tail (4 samples) evaluated eagerly."""
    from ddim_cold_amd.train import trainer as tr
    torch.manual_seed(0)
    model = build_model("vit_tiny").cuda().train()
    pool = synthetic_pool(1024, seed=4, device="cuda")
    idx = torch.randperm(1024)[:8 * 8 * 15 + 3 * 8 + 4]  # 15 groups of 8 batches + 3 batches + 4
    vals = {}
    for group in (8, 1):
        monkeypatch.setattr(tr, "EVAL_GROUP", group)
        eng = TrainEngine(model, EngineConfig(use_graph=True, temb_rows=7))
        rng = torch.tensor([123, 0], dtype=torch.int64, device="cuda")
        vals[group] = tr.evaluate(model, eng, pool, idx, 8, kind, 2000, rng)
        # one counter step per replay / eager batch
        assert int(rng[1]) == (15 + 3 + 1 if group == 8 else 8 * 15 + 3 + 1)
        eng.detach()
    assert abs(vals[8] - vals[1]) <= 0.05 * abs(vals[1]), vals


@pytest.mark.gpu
@pytest.mark.parametrize("draw", [True, False])
def test_gauss_batch_matches_reference_and_fused_embed(draw):
    """ops.gauss_batch (one launch: pool draw + randn + q_sample) == the CPU reference
    (same counter hash: t/idx exact, x_t to float rounding of the fast log/sincos), and
    the Gaussian mode of ops.patch_embed_cold_fwd == gauss_batch then patch_embed_fwd."""
    from ddim_cold_amd import ops
    from ddim_cold_amd.data.synthetic import SITE_DATA, SITE_NOISE
    from ddim_cold_amd.models.program import SITE_EMBED
    torch.manual_seed(0)
    model = build_model("vit_tiny").cuda().train()
    B, D, T = 8, model.embed_dim, model.total_steps
    N = model.patch_embed.num_patches + 1
    pool = synthetic_pool(32, seed=2, device="cuda")
    rng = torch.tensor([11, 5], dtype=torch.int64, device="cuda")
    idx0 = torch.randint(0, 32, (B,), device="cuda")

    def bufs(dev="cuda"):
        return (torch.empty(B, 3, 64, 64, device=dev), torch.empty(B, 3, 64, 64, device=dev),
                torch.empty(B, dtype=torch.int64, device=dev), idx0.clone().to(dev))

    xt, x0, t, idx = bufs()
    ops.gauss_batch(pool, rng, SITE_DATA, SITE_NOISE, T, xt, x0, t, idx, draw)
    cx, c0, ct, cidx = bufs("cpu")
    ops.gauss_batch(pool.cpu(), rng.cpu(), SITE_DATA, SITE_NOISE, T, cx, c0, ct, cidx, draw)
    torch.cuda.synchronize()
    assert torch.equal(t.cpu(), ct) and torch.equal(idx.cpu(), cidx) and torch.equal(x0.cpu(), c0)
    assert int(t.min()) >= 0 and int(t.max()) < T
    assert (xt.cpu() - cx).abs().max().item() < 2e-4
    # noise statistics over the batch: standard normal
    eps = (cx - c0 * torch.sqrt(1 - torch.sqrt((ct.double() + 1) / T)).float().view(-1, 1, 1, 1))
    eps = eps / torch.sqrt(torch.sqrt((ct.double() + 1) / T)).float().view(-1, 1, 1, 1)
    assert abs(eps.mean().item()) < 0.02 and abs(eps.std().item() - 1) < 0.02

    pe_w = model.patch_embed.proj.weight.detach().reshape(D, -1).to(torch.bfloat16).contiguous()
    args = (pe_w, model.patch_embed.proj.bias.detach(), model.cls_token.detach(), model.pos_embed.detach(),
            model.time_embed.weight.detach(), rng, SITE_EMBED, 0.1, model.patch_size)
    st = torch.empty(B * N, D // 32, 2, device="cuda")
    xb = torch.empty(B * N, D, dtype=torch.bfloat16, device="cuda")
    x_ref, p_ref = ops.patch_embed_fwd(xt, t, *args, ln_st=st, xb_out=xb)
    xt2, x02, t2, idx2 = bufs()
    st2, xb2 = torch.empty_like(st), torch.empty_like(xb)
    spec = (pool, SITE_DATA, 1, draw, True, x02, idx2, True, T, SITE_NOISE)
    x, p = ops.patch_embed_cold_fwd(spec, xt2, t2, *args, ln_st=st2, xb_out=xb2)
    torch.cuda.synchronize()
    assert torch.equal(t2, t) and torch.equal(idx2, idx) and torch.equal(x02, x0)
    assert (xt2 - xt).abs().max().item() <= 1e-6
    assert (p.float() - p_ref.float()).abs().max().item() <= 1e-2
    assert (x - x_ref).abs().max().item() <= 2e-2


@pytest.mark.gpu
def test_engine_gaussian_fused_batch_matches_unfused():
    """Gaussian DDIM training (t over the whole 2000-row table): the draw fused into the
    patch-embedding launch trains like the one-launch GaussianBatcher path."""
    from ddim_cold_amd.data.synthetic import GaussianBatcher

    def run(fuse):
        torch.manual_seed(0)
        model = build_model("vit_tiny").cuda().train()
        eng = TrainEngine(model, EngineConfig(lr=1e-3, t_max=100, seed=3, use_graph=True, graph_warmup=1,
                                              fuse_batch=fuse))
        eng.set_batch_fn(GaussianBatcher(synthetic_pool(64, seed=1, device="cuda"), 8, eng.rng, 2000))
        losses = [float(eng.train_step()) for _ in range(4)]
        torch.cuda.synchronize()
        return eng.flat_p.clone(), losses
    pf, lf = run(True)
    pu, lu = run(False)
    assert all(abs(a - b) <= 1e-3 * abs(b) for a, b in zip(lf, lu)), (lf, lu)
    assert (pf - pu).abs().max().item() <= 2 * 1e-3 * 4


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["cold", "cold_x0", "gaussian"])
def test_stepped_index_table_matches_explicit_rows(kind):
    """The trainer's device table (batch rows read at ``step counter % rows``, so K-step
    graphs need no host copy) draws the same batches as an explicit [B] index vector,
    for the fused patch-embedding draw and the stand-alone batch kernels."""
    from ddim_cold_amd import ops
    from ddim_cold_amd.data.synthetic import make_batcher
    torch.manual_seed(0)
    pool = synthetic_pool(40, seed=2, device="cuda")
    rows, A, B = 5, 2, 8
    table = torch.randint(0, 40, (rows, A, B), device="cuda")
    rng = torch.tensor([11, 3], dtype=torch.int64, device="cuda")
    ctr = torch.tensor([0, 7], dtype=torch.int64, device="cuda")  # step 7 -> row 2
    for j in range(A):
        want_idx = table[7 % rows, j].clone()
        st = make_batcher(kind, pool, B, rng, idx=table, idx_step=(ctr[1:2], j * B))
        ex = make_batcher(kind, pool, B, rng, idx=want_idx)
        a, b = st(), ex()
        torch.cuda.synchronize()
        assert all(torch.equal(u, v) for u, v in zip(a, b)), (kind, j)
        assert torch.equal(ops.stepped_idx(table, (ctr[1:2], j * B), B), want_idx)
        (xs, ts_, tt), spec = st.fused_spec()
        assert spec[10] is not None and spec[6] is table
    with pytest.raises(RuntimeError):  # a stepped table is read, never drawn into
        ops.cold_batch(pool, rng, 3, torch.empty(B, 3, 64, 64, device="cuda"), torch.empty(B, 3, 64, 64, device="cuda"),
                       torch.empty(B, dtype=torch.int64, device="cuda"), table, 6, True, idx_step=(ctr[1:2], 0))
    with pytest.raises(RuntimeError):  # batch offset past the end of a table row
        ops.cold_batch(pool, rng, 3, torch.empty(B, 3, 64, 64, device="cuda"), torch.empty(B, 3, 64, 64, device="cuda"),
                       torch.empty(B, dtype=torch.int64, device="cuda"), table, 6, False, idx_step=(ctr[1:2], A * B - 4))


@pytest.mark.gpu
def test_patch_embed_cold_stepped_table_matches_explicit():
    from ddim_cold_amd import ops
    from ddim_cold_amd.data.synthetic import SITE_DATA
    from ddim_cold_amd.models.program import SITE_EMBED
    torch.manual_seed(0)
    model = build_model("vit_tiny").cuda().train()
    B, D = 8, model.embed_dim
    N = model.patch_embed.num_patches + 1
    pool = synthetic_pool(32, seed=2, device="cuda")
    rng = torch.tensor([11, 5], dtype=torch.int64, device="cuda")
    table = torch.randint(0, 32, (3, 1, B), device="cuda")
    ctr = torch.tensor([4], dtype=torch.int64, device="cuda")  # row 1
    pe_w = model.patch_embed.proj.weight.detach().reshape(D, -1).to(torch.bfloat16).contiguous()
    args = (pe_w, model.patch_embed.proj.bias.detach(), model.cls_token.detach(), model.pos_embed.detach(),
            model.time_embed.weight.detach(), rng, SITE_EMBED, 0.1, model.patch_size)

    def run(idx, step):
        xt, tg = torch.empty(B, 3, 64, 64, device="cuda"), torch.empty(B, 3, 64, 64, device="cuda")
        t = torch.empty(B, dtype=torch.int64, device="cuda")
        st, xb = torch.empty(B * N, D // 32, 2, device="cuda"), torch.empty(B * N, D, dtype=torch.bfloat16, device="cuda")
        cold = (pool, SITE_DATA, 6, False, False, tg, idx, True, 0, 0, step)
        x, p = ops.patch_embed_cold_fwd(cold, xt, t, *args, ln_st=st, xb_out=xb)
        return x, p, xt, tg, t, st, xb
    a = run(table, (ctr, 0))
    b = run(table[1, 0].clone(), None)
    torch.cuda.synchronize()
    assert all(torch.equal(u, v) for u, v in zip(a, b))


@pytest.mark.gpu
@pytest.mark.parametrize("dataset", ["cold", "gauss"])
def test_embed_in_wgrad_launch_matches_separate_launch(monkeypatch, dataset):
    """engine.FUSE_EMBED_WGRAD (default): no embedding-backward launch -- the last
    LayerNorm backward writes the patch-row gradient, the cls / pos / time-embedding
    gradients and the LayerNorm finalize run inside the weight-gradient launch, each
    workgroup writing its own grad-norm partial -- == embed_bwd as its own launch (the
    same gradients; only the grad-norm partials are grouped differently), and two fused
    runs are bit-identical."""
    from ddim_cold_amd.data.synthetic import GaussianBatcher
    from ddim_cold_amd.train import engine as engine_mod

    def run(flag):
        monkeypatch.setattr(engine_mod, "FUSE_EMBED_WGRAD", flag)
        torch.manual_seed(0)
        model = build_model("vit_tiny").cuda().train()
        eng = TrainEngine(model, EngineConfig(lr=1e-3, t_max=100, seed=3, use_graph=True, graph_warmup=1,
                                              temb_rows=7 if dataset == "cold" else None))
        pool = synthetic_pool(64, seed=1, device="cuda")
        eng.set_batch_fn(ColdBatcher(pool, 16, eng.rng) if dataset == "cold" else
                         GaussianBatcher(pool, 16, eng.rng, 2000))
        losses = [float(eng.train_step()) for _ in range(4)]
        torch.cuda.synchronize()
        return eng.flat_p.clone(), losses
    pf, lf = run(True)
    pf2, lf2 = run(True)
    ps, ls = run(False)
    assert lf == lf2 and torch.equal(pf, pf2)
    assert all(abs(a - b) <= 1e-5 * abs(b) for a, b in zip(lf, ls)), (lf, ls)
    assert (pf - ps).abs().max().item() <= 1e-5


@pytest.mark.gpu
def test_transposed_weight_shadows_match_transposed_operand_path(monkeypatch):
    """Long-sequence models keep W^T shadows of the QKV / proj / fc1 weights
    (engine.TransposedShadows, refreshed after every optimizer step inside the graph) and
    run those input-gradient GEMMs on the k-contiguous path: same training as the
    transposed-operand path within the GEMMs' accumulation-order rounding, and the shadows
    equal the transposed bf16 weights after the run."""
    from ddim_cold_amd.train import engine as E

    def run(min_tokens):
        monkeypatch.setattr(E, "TRANSPOSED_DGRAD_MIN_TOKENS", min_tokens)
        torch.manual_seed(0)
        model = build_model("vit_small_200", depth=2).cuda().train()
        eng = TrainEngine(model, EngineConfig(lr=1e-3, t_max=100, seed=3, use_graph=True, graph_warmup=1,
                                              temb_rows=8, graph_steps=2))
        eng.set_batch_fn(ColdBatcher(synthetic_pool(32, (200, 200), seed=1, device="cuda"), 4, eng.rng))
        losses = [float(eng.train_steps(2)) for _ in range(2)]
        torch.cuda.synchronize()
        return eng, losses

    e1, l1 = run(512)
    assert e1.wt is not None and e1.param_tensors.blocks[0].qkv_wt is not None
    for bp in e1.param_tensors.blocks:
        for k in ("qkv", "proj", "fc1", "fc2"):
            assert torch.equal(getattr(bp, k + "_wt"), getattr(bp, k + "_w").t()), k
    e0, l0 = run(10 ** 9)
    assert e0.wt is None and e0.param_tensors.blocks[0].qkv_wt is None
    for a, b in zip(l1, l0):
        assert abs(a - b) <= 1e-4 * abs(b), (l1, l0)
    # Adam moves an element by ~lr per step whatever its gradient's size, so elements
    # with near-zero gradients may step differently under different rounding: bound the
    # largest difference by the 4 steps' reach and require almost all to agree closely
    d = (e1.flat_p - e0.flat_p).abs()
    assert d.max().item() <= 2 * 4 * 1e-3, d.max().item()
    assert (d > 1e-4).float().mean().item() < 0.01, (d > 1e-4).float().mean().item()


@pytest.mark.gpu
def test_transpose_bf16_op():
    from ddim_cold_amd import ops
    srcs = [torch.randn(r, c, device="cuda").to(torch.bfloat16) for r, c in ((1152, 384), (384, 384), (8, 72), (200, 136))]
    dsts = [torch.empty(s.shape[1], s.shape[0], dtype=torch.bfloat16, device="cuda") for s in srcs]
    ops.transpose_bf16_(srcs, dsts)
    for s, d in zip(srcs, dsts):
        assert torch.equal(d, s.t())
