"""Experiment layer on CPU: YAML config rules, trainer loop, log format, checkpoints, resume,
2-rank gloo training, CLI entry points."""
import dataclasses
import os
import subprocess
import sys

import pytest
import torch
import yaml

from ddim_cold_amd.config import ExperimentConfig, find_config, load_config
from ddim_cold_amd.train import checkpoint as ckpt
from ddim_cold_amd.train.trainer import Paths, launch
from ddim_cold_amd.utils.logging import parse_log

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_reference_config_rules():
    cfg = load_config(os.path.join(ROOT, "configs", "20220822.yaml")).validate()
    assert cfg.per_gpu_batch == 32  # AMP doubles the batch (multi_gpu_trainer.py:187-190)
    assert cfg.lr == pytest.approx(0.005 * 32 * 1 / 512)
    cfg8 = dataclasses.replace(cfg, num_gpus=8, AMP=False)
    assert cfg8.per_gpu_batch == 16 and cfg8.lr == pytest.approx(0.005 * 16 * 8 / 512)
    assert find_config("20220822").endswith("20220822.yaml")


def test_config_errors(tmp_path):
    p = tmp_path / "bad.yaml"
    p.write_text("batch_size: 4\nnot_a_key: 1\n")
    with pytest.raises(ValueError, match="not_a_key"):
        load_config(str(p))
    with pytest.raises(ValueError):
        ExperimentConfig(image_size=[64, 64], patch_size=7, synthetic=True).validate()
    with pytest.raises(ValueError):
        ExperimentConfig(dataStorage=["", ""]).validate()


def _tiny_cfg(**kw):
    base = dict(initializing="init.pkl", framework="_tiny", num_gpus=1, batch_size=4, epoch=[0, 2],
                image_size=[16, 16], patch_size=4, embed_dim=32, depth=2, head=2, synthetic=True,
                synthetic_size=64, log_every=2, graph=False)
    base.update(kw)
    return ExperimentConfig(**base).validate()


def test_trainer_log_checkpoints_and_resume(tmp_path):
    cfg = _tiny_cfg(ckpt_dir=str(tmp_path / "Saved_Models"))
    paths = Paths.make(cfg, "exp", root=str(tmp_path))
    res = launch(cfg, "exp", paths, backend="gloo")
    spe = 64 // 8
    assert res["steps"] == 2 * spe
    with open(paths.log) as f:
        text = f.read()
    assert text.startswith("Date: ") and f"TrainSet batchs:{spe}" in text and "TestSet batchs:1" in text
    steps, epochs = parse_log(paths.log)
    assert [s for s, _, _ in steps] == list(range(2, 2 * spe + 1, 2))
    assert [e for e, _ in epochs] == [0, 1]
    assert os.path.isfile(os.path.join(paths.saved_dir, "init.pkl"))
    last = torch.load(os.path.join(paths.ckpt_dir, "lastepoch.pkl"), weights_only=True)
    assert {"epoch", "steps", "loss_rec", "metric", "state_dict", "scheduler", "optimizer"} <= set(last)
    assert last["epoch"] == 1 and last["steps"] == 2 * spe
    assert all(k.startswith("module.") for k in last["state_dict"])
    assert last["scheduler"]["last_epoch"] == 2 * spe and last["scheduler"]["T_max"] == 2 * spe
    best = torch.load(os.path.join(paths.ckpt_dir, "bestloss.pkl"), weights_only=True)
    assert not any(k.startswith("module.") for k in best)
    opt = torch.optim.AdamW([torch.nn.Parameter(v.clone()) for v in best.values()])
    opt.load_state_dict(last["optimizer"])

    # resume: epoch+1, steps continue, optimizer/scheduler restored
    cfg2 = dataclasses.replace(cfg, resume=os.path.join(paths.ckpt_dir, "lastepoch.pkl"), epoch=[0, 3])
    res2 = launch(cfg2, "exp", paths, backend="gloo")
    assert res2["steps"] == 3 * spe
    assert [e for e, _ in res2["history"]] == [2]
    with open(paths.log) as f:
        text = f.read()
    assert "resuming from epoch        2 of" in text and "recovering best_loss" in text
    last2 = torch.load(os.path.join(paths.ckpt_dir, "lastepoch.pkl"), weights_only=True)
    assert float(last2["optimizer"]["state"][0]["step"]) == 3 * spe


def test_trainer_grad_accum(tmp_path):
    cfg = _tiny_cfg(grad_accum=2, epoch=[0, 1], ckpt_dir=str(tmp_path / "Saved_Models"))
    paths = Paths.make(cfg, "acc", root=str(tmp_path))
    res = launch(cfg, "acc", paths, backend="gloo")
    assert res["steps"] == 64 // (8 * 2)
    last = torch.load(os.path.join(paths.ckpt_dir, "lastepoch.pkl"), weights_only=True)
    assert float(last["optimizer"]["state"][0]["step"]) == res["steps"]


def test_fault_injection_and_resume(tmp_path):
    from ddim_cold_amd.utils.observe import FaultInjected
    cfg = _tiny_cfg(ckpt_dir=str(tmp_path / "Saved_Models"), fault_inject_step=10, sync_check_every=3)
    paths = Paths.make(cfg, "flt", root=str(tmp_path))
    with pytest.raises(FaultInjected):
        launch(cfg, "flt", paths, backend="gloo")
    last = torch.load(os.path.join(paths.ckpt_dir, "lastepoch.pkl"), weights_only=True)
    assert last["epoch"] == 0 and last["steps"] == 8 and last["scaler"]["scale"] == 1.0
    cfg2 = dataclasses.replace(cfg, fault_inject_step=0, resume=os.path.join(paths.ckpt_dir, "lastepoch.pkl"))
    res = launch(cfg2, "flt", paths, backend="gloo")
    assert res["steps"] == 16 and [e for e, _ in res["history"]] == [1]
    with open(paths.log) as f:
        assert "# perf:" in f.read()


def test_checkpoint_weights_roundtrip(tmp_path):
    from ddim_cold_amd.models import DiffusionVisionTransformer
    m = DiffusionVisionTransformer(img_size=[16, 16], patch_size=4, embed_dim=32, depth=1, num_heads=2)
    p = str(tmp_path / "w.pkl")
    ckpt.save_weights(m, p)
    m2 = DiffusionVisionTransformer(img_size=[16, 16], patch_size=4, embed_dim=32, depth=1, num_heads=2)
    ckpt.load_weights(m2, p)
    assert all(torch.equal(a, b) for a, b in zip(m.state_dict().values(), m2.state_dict().values()))
    # DDP-prefixed dict and lastepoch-style dict both load
    torch.save({"state_dict": ckpt.add_prefix(m.state_dict()), "epoch": 3}, p)
    ckpt.load_weights(m2, p)


def test_plumbing_config_gaussian32(tmp_path):
    """BASELINE.json config #1: full-size ViT-tiny on 32x32 synthetic Gaussian-diffusion
    images, batch 8, one gloo rank on the CPU, from the shipped YAML."""
    cfg = load_config(os.path.join(ROOT, "configs", "plumbing_gaussian32.yaml")).validate()
    assert (cfg.dataset, cfg.image_size, cfg.per_gpu_batch, cfg.embed_dim, cfg.depth) == \
        ("gaussian", [32, 32], 8, 384, 7)
    cfg = dataclasses.replace(cfg, ckpt_dir=str(tmp_path / "Saved_Models"))
    paths = Paths.make(cfg, "plumbing_gaussian32", root=str(tmp_path))
    res = launch(cfg, "plumbing_gaussian32", paths, backend="gloo")
    assert res["steps"] == 64 // 8
    steps, epochs = parse_log(paths.log)
    assert len(epochs) == 1 and 0 < epochs[0][1] < 10
    assert all(loss == loss for _, loss, _ in steps)  # finite EMA losses
    last = torch.load(os.path.join(paths.ckpt_dir, "lastepoch.pkl"), weights_only=True)
    assert last["state_dict"]["module.pos_embed"].shape[1] == (32 // 8) ** 2 + 1


def test_trainer_two_ranks_gloo(tmp_path):
    cfg = _tiny_cfg(num_gpus=2, epoch=[0, 1], ckpt_dir=str(tmp_path / "Saved_Models"), sync_check_every=2)
    paths = Paths.make(cfg, "exp2", root=str(tmp_path))
    res = launch(cfg, "exp2", paths, backend="gloo")
    assert res["steps"] == 64 // 2 // 8
    steps, epochs = parse_log(paths.log)
    assert len(epochs) == 1 and epochs[0][1] > 0


def test_two_rank_resume_keeps_per_rank_seeds(tmp_path):
    """lastepoch.pkl is written by rank 0; a 2-rank resume must keep each rank's own
    RNG seed (independent cold t / dropout draws) and restore only the step counter."""
    cfg = _tiny_cfg(num_gpus=2, epoch=[0, 1], ckpt_dir=str(tmp_path / "Saved_Models"))
    paths = Paths.make(cfg, "res2", root=str(tmp_path))
    res = launch(cfg, "res2", paths, backend="gloo")
    seeds = {r: v["rng"][0] for r, v in res["per_rank"].items()}
    assert len(seeds) == 2 and seeds[0] != seeds[1]
    cfg2 = dataclasses.replace(cfg, resume=os.path.join(paths.ckpt_dir, "lastepoch.pkl"), epoch=[0, 2])
    res2 = launch(cfg2, "res2", paths, backend="gloo")
    pr = res2["per_rank"]
    assert {r: v["rng"][0] for r, v in pr.items()} == seeds
    # step counter continued from the checkpoint on every rank
    assert pr[0]["rng"][1] == pr[1]["rng"][1] == 2 * res["per_rank"][0]["rng"][1]
    # eval draws differ per rank and follow the epoch
    assert pr[0]["eval_rng"][0] != pr[1]["eval_rng"][0]
    nvb = res["per_rank"][0]["eval_rng"][1]  # val batches per rank (epoch 0 evaluated)
    assert nvb >= 1 and pr[0]["eval_rng"][1] == pr[1]["eval_rng"][1] == 2 * nvb


def test_cli_entry_points(tmp_path):
    cfg = dict(initializing="init.pkl", framework="_cli", num_gpus=1, batch_size=4, epoch=[0, 1],
               image_size=[16, 16], patch_size=4, embed_dim=32, depth=1, head=2, synthetic=True,
               synthetic_size=32, log_every=100, graph=False, dataStorage=["", ""])
    p = tmp_path / "cliexp.yaml"
    p.write_text(yaml.safe_dump(cfg))
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "multi_gpu_trainer.py"), str(p), "--root", str(tmp_path),
                        "--backend", "gloo"], capture_output=True, text=True, env=env, timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-2000:]
    log = tmp_path / "Saved_Models" / "cliexp_cli" / "train.log"
    assert log.is_file() and (tmp_path / "Saved_Models" / "cliexp_cli" / "cliexp.yaml").is_file()
    w = tmp_path / "Saved_Models" / "cliexp_cli" / "lastepoch.pkl"
    out = tmp_path / "out"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "ViT.py"), "--model", "oxford_flower", "--sample_n", "2",
                        "--acc_k", "400", "--seq_n", "1", "--seq_k", "500", "--out_dir", str(out)],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert any(f.endswith(".png") for f in os.listdir(out))
    assert w.is_file()


def test_trainer_stops_on_comm_error(tmp_path, monkeypatch):
    """The trainer checks the data-parallel hand-off at every log point
    (TrainEngine.check_comm) and a failure ends the run with an error."""
    from ddim_cold_amd.train import engine as eng_mod
    calls = []

    def failing_check(self):
        calls.append(1)
        raise RuntimeError("data-parallel hand-off: a comm-stream flag wait timed out (test)")
    monkeypatch.setattr(eng_mod.TrainEngine, "check_comm", failing_check)
    cfg = _tiny_cfg(ckpt_dir=str(tmp_path / "Saved_Models"))
    paths = Paths.make(cfg, "exp", root=str(tmp_path))
    with pytest.raises(RuntimeError, match="hand-off"):
        launch(cfg, "exp", paths, backend="gloo")
    assert len(calls) == 1
    assert not os.path.exists(os.path.join(paths.ckpt_dir, "lastepoch.pkl"))  # nothing saved after it


def test_async_lastepoch_equals_sync_and_resumes_identically(tmp_path):
    """lastepoch.pkl written by the background CheckpointWriter (host snapshot) holds
    exactly what the synchronous write holds, and resuming from either gives the
    same training state."""
    from ddim_cold_amd.data.synthetic import ColdBatcher, synthetic_pool
    from ddim_cold_amd.models import DiffusionVisionTransformer
    from ddim_cold_amd.train.engine import EngineConfig, TrainEngine

    def make():
        torch.manual_seed(3)
        m = DiffusionVisionTransformer(img_size=[16, 16], patch_size=4, embed_dim=32, depth=2, num_heads=2)
        e = TrainEngine(m, EngineConfig(lr=1e-3, t_max=20, use_graph=False, seed=9, temb_rows=5), device="cpu")
        e.set_batch_fn(ColdBatcher(synthetic_pool(16, size=(16, 16), seed=1), 4, e.rng))
        return m, e

    m, e = make()
    for _ in range(3):
        e.train_step()
    sync_p, async_p = str(tmp_path / "sync.pkl"), str(tmp_path / "async.pkl")
    best_p = str(tmp_path / "best.pkl")
    ckpt.save_lastepoch(sync_p, m, e, 0, 3, 0.5, 0.25)
    w = ckpt.CheckpointWriter()
    w.submit(e.snapshot_to_host(), async_p, 0, 3, 0.5, 0.25, best_path=best_p)
    e.train_step()  # training goes on while the file is written; the snapshot is unaffected
    w.join()
    a = torch.load(sync_p, weights_only=True)
    b = torch.load(async_p, weights_only=True)
    assert a.keys() == b.keys()

    def eq(x, y):
        if torch.is_tensor(x):
            return torch.equal(x, y)
        if isinstance(x, dict):
            return x.keys() == y.keys() and all(eq(x[k], y[k]) for k in x)
        if isinstance(x, (list, tuple)):
            return len(x) == len(y) and all(eq(u, v) for u, v in zip(x, y))
        return x == y
    assert eq(a, b)
    assert eq(ckpt.strip_prefix(a["state_dict"]), torch.load(best_p, weights_only=True))
    finals = []
    for path in (sync_p, async_p):
        m2, e2 = make()
        ckpt.load_lastepoch(path, m2, e2)
        for _ in range(2):
            e2.train_step()
        finals.append((e2.flat_p.clone(), e2.flat_m.clone(), e2.step_ctr.clone()))
    assert all(torch.equal(x, y) for x, y in zip(*finals))


def test_back_to_back_snapshots_do_not_tear_a_slow_write(tmp_path, monkeypatch):
    """A second epoch-end submit while the first write is still laying out its file
    must not overwrite the snapshot buffers under it (the trainer passes the snapshot
    callable, which the writer calls only after joining the previous write)."""
    import time
    from ddim_cold_amd.data.synthetic import ColdBatcher, synthetic_pool
    from ddim_cold_amd.models import DiffusionVisionTransformer
    from ddim_cold_amd.train.engine import EngineConfig, TrainEngine

    torch.manual_seed(3)
    m = DiffusionVisionTransformer(img_size=[16, 16], patch_size=4, embed_dim=32, depth=2, num_heads=2)
    e = TrainEngine(m, EngineConfig(lr=1e-2, t_max=20, use_graph=False, seed=9, temb_rows=5), device="cpu")
    e.set_batch_fn(ColdBatcher(synthetic_pool(16, size=(16, 16), seed=1), 4, e.rng))
    for _ in range(2):
        e.train_step()
    want = {k: v.clone() for k, v in m.state_dict().items()}
    real = ckpt.lastepoch_dict
    calls = []

    def slow_layout(snap, *a):
        calls.append(1)
        if len(calls) == 1:
            time.sleep(0.5)  # the first write is still reading its snapshot...
        return real(snap, *a)
    monkeypatch.setattr(ckpt, "lastepoch_dict", slow_layout)
    w = ckpt.CheckpointWriter()
    p1, p2 = str(tmp_path / "e0.pkl"), str(tmp_path / "e1.pkl")
    w.submit(e.snapshot_to_host, p1, 0, 2, 0.5, 0.25)
    for _ in range(3):  # ...when the next epoch ends and snapshots again
        e.train_step()
    w.submit(e.snapshot_to_host, p2, 1, 5, 0.4, 0.2)
    w.join()
    got = ckpt.strip_prefix(torch.load(p1, weights_only=True)["state_dict"])
    assert all(torch.equal(got[k], want[k]) for k in want)
    later = ckpt.strip_prefix(torch.load(p2, weights_only=True)["state_dict"])
    assert any(not torch.equal(later[k], want[k]) for k in want)


def test_checkpoint_writer_surfaces_errors(tmp_path):
    class Bad:
        def wait(self):
            raise OSError("disk full (test)")
    w = ckpt.CheckpointWriter()
    w.submit(Bad(), str(tmp_path / "x.pkl"), 0, 0, 0.0, 0.0)
    with pytest.raises(RuntimeError, match="disk full"):
        w.join()
    w.join()  # reported once


def test_is_capture_error_matches_capture_failures_only():
    from ddim_cold_amd.utils.observe import is_capture_error
    assert is_capture_error(RuntimeError("HIP error: operation not permitted when stream is capturing"))
    assert is_capture_error(RuntimeError("hipErrorStreamCaptureInvalidated: capture invalidated"))
    # the runtime's hipGetErrorString texts (what torch reports)
    for msg in ("operation failed due to a previous error during capture", "capturing stream has unjoined work",
                "dependency created on uncaptured work in another stream",
                "operation not permitted on an event last recorded in a capturing stream"):
        assert is_capture_error(RuntimeError(f"HIP error: {msg}")), msg
    # real errors that merely mention a graph are not swallowed into the eager fallback
    assert not is_capture_error(RuntimeError("shape mismatch in graph input buffer"))
    assert not is_capture_error(RuntimeError("HIP error: an illegal memory access was encountered"))
    assert not is_capture_error(ValueError("hipErrorStreamCaptureInvalidated"))


def test_reference_l5_api_shims(tmp_path):
    """multi_gpu_trainer's library functions with the reference signatures
    (multi_gpu_trainer.py:18-51): evaluate() over a torch DataLoader of
    ColdDownSampleDataset batches equals the per-batch mean smooth-L1, and main(rank,
    world_size, ...) trains one rank into the reference's log / checkpoint files."""
    import importlib.util
    import numpy as np
    from PIL import Image
    from torch.utils.data import DataLoader
    from ddim_cold_amd.data.datasets import ColdDownSampleDataset
    from ddim_cold_amd.models import DiffusionVisionTransformer
    spec = importlib.util.spec_from_file_location("mgt", os.path.join(ROOT, "multi_gpu_trainer.py"))
    mgt = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mgt)
    for d in ("train", "val"):
        os.makedirs(tmp_path / d)
        g = np.random.default_rng(3 if d == "train" else 4)
        for i in range(12):
            Image.fromarray(g.integers(0, 255, (20, 20, 3), dtype=np.uint8)).save(tmp_path / d / f"{i}.png")
    torch.manual_seed(0)
    model = DiffusionVisionTransformer(img_size=[16, 16], patch_size=4, embed_dim=32, depth=2, num_heads=2)
    ds = ColdDownSampleDataset(str(tmp_path / "val"), imgSize=[16, 16])
    loader = DataLoader(ds, batch_size=4, shuffle=False)
    import random
    random.seed(5)
    np.random.seed(5)
    torch.manual_seed(5)  # the dataset draws each sample's t at random
    got = mgt.evaluate(model, loader, "cpu")
    assert not model.training
    want = []
    random.seed(5)
    np.random.seed(5)
    torch.manual_seed(5)
    with torch.no_grad():
        for x, y, t in loader:
            want.append(torch.nn.functional.smooth_l1_loss(model(x, t), y).item())
    assert got == pytest.approx(float(np.array(want).mean()), rel=1e-6)
    log = str(tmp_path / "Saved_Models" / "exp" / "train.log")
    os.makedirs(os.path.dirname(log), exist_ok=True)
    mgt.printLog("hello", log)
    res = mgt.main(0, 1, "init.pkl", True, 4, [0, 1], 1e-3, "none",
                   [str(tmp_path / "train"), str(tmp_path / "val")], str(tmp_path / "Saved_Models") + "/", log,
                   str(tmp_path / "Saved_Models" / "exp") + "/", [16, 16], 4, 4, 32, 2, 2,
                   backend="gloo", graph=False, log_every=1, num_workers=0)
    assert res["steps"] == 3  # 12 images // batch 4
    text = open(log).read()
    assert text.startswith("hello\nDate: ") and "TrainSet batchs:3" in text and "epoch:    0" in text
    assert os.path.isfile(tmp_path / "Saved_Models" / "init.pkl")
    ck = torch.load(tmp_path / "Saved_Models" / "exp" / "lastepoch.pkl", weights_only=True)
    assert ck["steps"] == 3 and ck["scheduler"]["base_lrs"] == [pytest.approx(1e-3)]


def test_epoch_table_rotation_keeps_sampler_order_for_any_start_counter():
    """The trainer's device step table is rotated by the epoch's starting scheduler
    counter, so step j of the epoch reads DistributedSampler batch j even when a resume
    left the counter at a non-multiple of steps_per_epoch (trainer.py epoch start)."""
    from ddim_cold_amd import ops
    spe, A, B = 5, 1, 3
    table = torch.arange(spe * A * B, dtype=torch.int64).view(spe, A, B)
    for start in (0, 5, 7, 13):
        dev_table = table.roll(start % spe, 0)
        for j in range(spe):
            ctr = torch.tensor([start + j])
            got = ops.stepped_idx(dev_table, (ctr, 0), B)
            assert torch.equal(got, table[j, 0]), (start, j)
