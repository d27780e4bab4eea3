"""Data parallel at the target world sizes without a multi-GPU node: 4 and 8 gloo
ranks on the CPU (the same engine / trainer / bench code paths the RCCL job runs;
multi_gpu_trainer.py:61-62, :88, :141-146, :212-219 are the reference counterparts).

* engine: every gradient-exchange layout (overlap-1/2/3/7, inline-1), fp32 and bf16
  wire, cold (inactive time_embed rows skipped) and Gaussian (sparse time_embed
  (t, row) all-gather) == one process on the concatenated batch;
* ``bench.py --gpus 8`` self-spawn: one JSON line, n_gpus 8 / dp8;
* an 8-rank trainer run + resume, with a validation set that 8 does not divide
  (DistributedSampler padding);
* one rank failing mid-epoch ends ``launch()`` with an error naming it."""
import json
import os
import tempfile
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ddim_cold_amd.models import DiffusionVisionTransformer
from ddim_cold_amd.parallel.dist import free_port
from ddim_cold_amd.train.engine import EngineConfig, TrainEngine

CFG = dict(img_size=[16, 16], patch_size=4, embed_dim=32, depth=7, num_heads=2)
GB = 8  # global batch
VARIANTS = [  # (name, wire, gaussian, layout)
    ("fp32-cold-overlap-1", "fp32", False, "overlap-1"),
    ("fp32-cold-overlap-2", "fp32", False, "overlap-2"),
    ("fp32-cold-overlap-3", "fp32", False, "overlap-3"),
    ("fp32-cold-overlap-7", "fp32", False, "overlap-7"),
    ("fp32-cold-inline-1", "fp32", False, "inline-1"),
    ("bf16-cold-overlap-2", "bf16", False, "overlap-2"),
    ("fp32-gauss-overlap-2", "fp32", True, "overlap-2"),
    ("fp32-gauss-inline-1", "fp32", True, "inline-1"),
    ("bf16-gauss-overlap-3", "bf16", True, "overlap-3"),
]


def _model(seed):
    torch.manual_seed(seed)
    return DiffusionVisionTransformer(**CFG, drop_rate=0.0, attn_drop_rate=0.0, drop_path_rate=0.0).train()


def _batch(gauss):
    g = torch.Generator().manual_seed(5)
    x = torch.randn(GB, 3, 16, 16, generator=g)
    y = torch.randn(GB, 3, 16, 16, generator=g).clamp(-1, 1)
    t = torch.randint(0, 2000, (GB,), generator=g)
    if gauss:  # repeats within one rank's slice (at world 4) and across ranks
        return x, y, t[[0, 0, 1, 0, 2, 3, 1, 4]]
    return x, y, t % 6 + 1


def _engine(wire, gauss, seed):
    return TrainEngine(_model(seed), EngineConfig(lr=1e-3, weight_decay=0.0, max_grad_norm=0.0, grad_wire=wire,
                                                  temb_rows=None if gauss else 7), device="cpu")


def _world_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b = GB // world
        res = {}
        for name, wire, gauss, layout in VARIANTS:
            eng = _engine(wire, gauss, seed=rank)  # different init per rank: rank 0's is broadcast
            eng.apply_layout(layout)
            assert (eng.temb_bucket is not None) == (gauss and layout != "inline-1") or gauss
            x, y, t = _batch(gauss)
            sl = slice(rank * b, (rank + 1) * b)
            eng.step(x[sl], y[sl], t[sl])
            m = eng.flat_m.clone()
            ms = [torch.zeros_like(m) for _ in range(world)]
            dist.all_gather(ms, m)
            res[name] = (m, all(torch.equal(ms[0], q) for q in ms), len(eng.buckets))
        if rank == 0:
            torch.save(res, out_path)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [4, 8])
def test_data_parallel_world_matches_single_process(world):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r.pt")
        mp.start_processes(_world_worker, args=(world, free_port(), out), nprocs=world, join=True,
                           start_method="spawn")
        res = torch.load(out, weights_only=True)
    refs = {}
    for gauss in (False, True):
        eng = _engine("fp32", gauss, seed=0)
        eng.step(*_batch(gauss))
        refs[gauss] = (eng.flat_m.clone(), eng.offsets["time_embed.weight"])
    for name, wire, gauss, layout in VARIANTS:
        m, same, nb = res[name]
        assert same, f"{name}: replicas differ"
        m1, (o, k) = refs[gauss]
        tol = 1e-4 if wire == "fp32" else 2e-2
        err = (m - m1).abs().max().item() / m1.abs().max().item()
        assert err < tol, (name, err)
        te, te1 = m[o:o + k], m1[o:o + k]
        assert te1.abs().max() > 0 and (te - te1).abs().max().item() <= tol * te1.abs().max().item(), name
        if layout == "inline-1":
            assert nb == 1
        else:
            blocks = int(layout.split("-")[1])
            assert nb == -(-7 // blocks) + 1, (name, nb)  # block buckets + the embedding bucket


def test_bench_self_spawn_eight_ranks_cpu():
    from test_bench_cpu import REQUIRED, _bench
    r = _bench(["--gpus", "8", "--steps", "1", "--warmup", "1", "--no-sampler", "--batch", "4"], timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert REQUIRED <= set(out)
    assert out["n_gpus"] == 8 and out["config"]["parallelism"] == "dp8"
    assert out["config"]["global_batch"] == 32 and out["config"]["launcher"] == "self-spawn"
    assert out["value"] > 0 and out["scaling"] == "weak"


def _tiny_cfg(**kw):
    from ddim_cold_amd.config import ExperimentConfig
    base = dict(initializing="init.pkl", framework="_w8", num_gpus=8, batch_size=4, epoch=[0, 1],
                image_size=[16, 16], patch_size=4, embed_dim=32, depth=2, head=2, synthetic=True,
                synthetic_size=136, log_every=1, graph=False)
    base.update(kw)
    return ExperimentConfig(**base).validate()


def test_trainer_eight_ranks_resume_and_padded_val(tmp_path):
    from ddim_cold_amd.data.datasets import shard_indices
    from ddim_cold_amd.train.trainer import Paths, launch
    from ddim_cold_amd.utils.logging import parse_log
    cfg = _tiny_cfg(ckpt_dir=str(tmp_path / "Saved_Models"))
    n_val = 136 // 8  # 17 validation images: 8 ranks x 3 after padding with 7 duplicates
    shards = [shard_indices(n_val, 8, r, 0, cfg.seed, shuffle=False, drop_last=False) for r in range(8)]
    assert all(s.numel() == 3 for s in shards) and sum(s.numel() for s in shards) == 24
    assert sorted(set(torch.cat(shards).tolist())) == list(range(n_val))
    paths = Paths.make(cfg, "w8", root=str(tmp_path))
    res = launch(cfg, "w8", paths, backend="gloo")
    pr = res["per_rank"]
    assert sorted(pr) == list(range(8))
    spe = (136 // 8) // cfg.per_gpu_batch  # DistributedSampler(drop_last) shard // batch
    assert res["steps"] == spe
    assert len({v["rng"][0] for v in pr.values()}) == 8  # independent per-rank draws
    assert all(v["eval_rng"][1] == 1 for v in pr.values())  # one (ragged, padded) val batch per rank
    assert len({round(v["history"][0][1], 6) for v in pr.values()}) == 1  # all-reduced val loss
    steps, epochs = parse_log(paths.log)
    assert [e for e, _ in epochs] == [0] and epochs[0][1] > 0
    cfg2 = _tiny_cfg(ckpt_dir=str(tmp_path / "Saved_Models"), epoch=[0, 2],
                     resume=os.path.join(paths.ckpt_dir, "lastepoch.pkl"))
    res2 = launch(cfg2, "w8", paths, backend="gloo")
    pr2 = res2["per_rank"]
    assert res2["steps"] == 2 * spe and all(v["rng"][1] == 2 * pr[0]["rng"][1] for v in pr2.values())
    assert {r: v["rng"][0] for r, v in pr2.items()} == {r: v["rng"][0] for r, v in pr.items()}
    assert [e for e, _ in res2["history"]] == [1]


def test_one_rank_failing_mid_epoch_stops_launch(tmp_path):
    from ddim_cold_amd.train.trainer import Paths, launch
    cfg = _tiny_cfg(ckpt_dir=str(tmp_path / "Saved_Models"), synthetic_size=400, fault_inject_step=2,
                    fault_inject_rank=5)
    paths = Paths.make(cfg, "w8f", root=str(tmp_path))
    t0 = time.time()
    with pytest.raises(RuntimeError, match="rank5"):
        launch(cfg, "w8f", paths, backend="gloo")
    assert time.time() - t0 < 300
    assert not os.path.exists(os.path.join(paths.ckpt_dir, "lastepoch.pkl"))
