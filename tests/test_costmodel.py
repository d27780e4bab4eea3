"""All-reduce cost model + bucket plan (parallel/costmodel.py) and the engine hooks
that use it (layout names, model-ordered autotune candidates)."""
import math

import pytest

from ddim_cold_amd.parallel import costmodel as cm


def test_fit_recovers_alpha_and_bandwidth():
    true = cm.AllReduceModel(8, 25.0, 400.0)
    sizes = [2 ** k for k in range(18, 26)]
    m = cm.fit_allreduce(8, sizes, [true.time_us(s) for s in sizes])
    assert abs(m.alpha_us - 25.0) < 1e-6 and abs(m.algbw_gbs - 400.0) < 1e-6
    assert abs(m.busbw_gbs - 400.0 * 2 * 7 / 8) < 1e-6
    # noisy small sizes with a negative intercept: bandwidth-only fit through the largest
    m2 = cm.fit_allreduce(2, [1e5, 1e6], [1.0, 20.0])
    assert m2.alpha_us == 0.0 and abs(m2.time_us(1e6) - 20.0) < 1e-9


def test_xgmi_ring_model_scales_with_links():
    big = 64 << 20
    t2 = cm.xgmi_ring_model(2).time_us(big) - cm.xgmi_ring_model(2).alpha_us
    t8 = cm.xgmi_ring_model(8).time_us(big) - cm.xgmi_ring_model(8).alpha_us
    # N-1 links in parallel: the per-byte cost at 2 ranks (one link) is 4x that at 8
    assert abs(t2 / t8 - 4.0) < 1e-9
    assert cm.xgmi_ring_model(1).time_us(big) == 0.0
    with pytest.raises(ValueError):
        cm.xgmi_ring_model(9)


def _prof():
    return cm.vit_step_profile(7, 384, 384, 2080, 176_832)


def test_simulate_inline_and_overlap_limits():
    p = _prof()
    m = cm.xgmi_ring_model(8)
    total = 7 * p.block_bytes + p.embed_bytes
    r = cm.simulate_step(p, m, 1, inline=True)
    assert r["exposed_us"] == pytest.approx(m.time_us(total)) and r["buckets"] == 1
    # free collectives: only the extra bucket launches are exposed
    free = cm.AllReduceModel(8, 0.0, math.inf)
    for bb in (1, 2, 7):
        r = cm.simulate_step(p, free, bb)
        nb = math.ceil(7 / bb) + 1
        assert r["buckets"] == nb
        assert r["exposed_us"] == pytest.approx(nb * p.bucket_overhead_us)
    # collectives slower than the backward: the comm queue is the critical path
    slow = cm.AllReduceModel(8, 0.0, 1.0)
    r = cm.simulate_step(p, slow, 1)
    assert r["exposed_us"] > r["comm_us"] - r["bwd_us"]


def test_plan_orders_layouts_and_prefers_overlap_on_one_link():
    p = _prof()
    plan = cm.plan_buckets(p, cm.xgmi_ring_model(2))
    assert [x[4] for x in plan] == sorted(x[4] for x in plan)
    assert plan[0][0].startswith("overlap-")  # 2 ranks share one link: overlap pays
    names = {x[0] for x in plan}
    assert names == {f"overlap-{k}" for k in range(1, 8)} | {"inline-1"}
    assert "| 8 |" in cm.describe(p)


def test_engine_layout_names_and_model_candidates():
    from ddim_cold_amd import build_model
    from ddim_cold_amd.config import ExperimentConfig
    from ddim_cold_amd.train.engine import EngineConfig, TrainEngine
    assert TrainEngine.layout_by_name("overlap-3") == ("overlap-3", 3, True, False)
    assert TrainEngine.layout_by_name("inline-1")[3] is True
    with pytest.raises(ValueError):
        TrainEngine.layout_by_name("overlap-0")
    eng = TrainEngine(build_model("vit_tiny"), EngineConfig(lr=1e-3, t_max=10, temb_rows=7, use_graph=False),
                      device="cpu")
    prof = eng.step_profile()
    assert prof.block_bytes == 4 * 887_040  # the four Linears; LayerNorms sit in the last bucket
    assert 7 * prof.block_bytes + prof.embed_bytes + prof.head_bytes == pytest.approx(4 * eng.reduced_numel())
    # the simulator's per-bucket bytes are the engine's own bucket ranges, for every layout
    for bb in (1, 2, 3, 4, 7):
        for eb in (True, False):
            eng.set_comm_layout(bb, eb)
            got = [4 * sum(b - a for a, b in rs) for rs in eng.bucket_ranges]
            want = [nb for _, nb in cm.bucket_plan(prof, bb, eb)]
            assert got == pytest.approx(want), (bb, eb)
    eng.world = 2
    cands = eng.candidate_layouts()
    assert {L[0] for L in TrainEngine.COMM_LAYOUTS} <= {L[0] for L in cands}
    best = eng.model_layouts()[0][0]
    assert best in {L[0] for L in cands} and all(len(L) == 4 for L in cands)
    assert cands[0][0] == "graph-inline-1"  # the captured inline layout is measured first
    assert TrainEngine.layout_by_name("graph-inline-1") == ("graph-inline-1", 1 << 16, False, True)
    assert TrainEngine.layout_by_name("graph-overlap-4") == ("graph-overlap-4", 4, True, False)
    cfg = ExperimentConfig(synthetic=True, comm_layout="overlap-5")
    assert cfg.validate() is cfg
    with pytest.raises(ValueError):
        ExperimentConfig(synthetic=True, comm_layout="overlap-x").validate()


def _probe_worker(rank, world, port, q):
    import os
    import torch.distributed as dist
    from ddim_cold_amd import build_model
    from ddim_cold_amd.train.engine import EngineConfig, TrainEngine
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        eng = TrainEngine(build_model("vit_tiny"), EngineConfig(lr=1e-3, t_max=10, temb_rows=7, use_graph=False),
                          device="cpu")
        fit, probe = eng.probe_allreduce(sizes_mb=(0.0625, 0.25, 1.0), reps=2)
        q.put((rank, fit.alpha_us, fit.algbw_gbs, sorted(probe), eng.candidate_layouts()[0][0]))
    finally:
        dist.destroy_process_group()


def test_probe_allreduce_gloo_two_ranks():
    """probe_allreduce measures the engine's own collective path on every rank and all
    ranks end up with the same (max-reduced) fit and the same model-ordered candidates."""
    import torch.multiprocessing as mp
    from ddim_cold_amd.parallel.dist import free_port
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_probe_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, a0, b0, s0, c0), (_, a1, b1, s1, c1) = res
    assert s0 == s1 == [4 * (1 << 14), 4 * (1 << 16), 4 * (1 << 18)]
    assert (a0, b0, c0) == (a1, b1, c1) and a0 >= 0 and b0 > 0
