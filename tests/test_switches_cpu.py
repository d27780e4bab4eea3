"""Every remaining DDIM_COLD_* environment switch has a test (README "Environment
switches" lists them).  The ones that need a GPU are exercised by GPU tests:
DDIM_COLD_FAKE_COMM, DDIM_COLD_TEST_HANDOFF_SKEW and DDIM_COLD_HANDOFF_TIMEOUT_US by
tests/test_trainer_overlap_gpu.py."""
import json
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _py(code, env=None, timeout=300):
    e = dict(os.environ, PYTHONPATH=ROOT)
    for k in list(e):
        if k.startswith("DDIM_COLD_"):
            e.pop(k)
    e.update(env or {})
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=timeout, env=e,
                          cwd=ROOT)


class _FakeCuda:
    is_cuda = True


def test_allow_reference_policy(monkeypatch):
    """A GPU tensor with no loadable extension: NativeExtensionError, unless
    DDIM_COLD_ALLOW_REFERENCE=1 routes it to the PyTorch reference ops."""
    from ddim_cold_amd.ops import _ext
    monkeypatch.setattr(_ext, "LIB_PATH", "/nonexistent/_C.so")
    monkeypatch.setattr(_ext, "_STATE", {"loaded": False, "error": None, "path": None})
    monkeypatch.delenv("DDIM_COLD_ALLOW_REFERENCE", raising=False)
    with pytest.raises(_ext.NativeExtensionError, match="ALLOW_REFERENCE"):
        _ext.require_for(_FakeCuda())
    monkeypatch.setenv("DDIM_COLD_ALLOW_REFERENCE", "1")
    assert _ext.require_for(_FakeCuda()) is False


def test_force_reference_model_forward(monkeypatch):
    from ddim_cold_amd.models import vit
    monkeypatch.delenv("DDIM_COLD_FORCE_REFERENCE", raising=False)
    assert vit._fused_allowed(_FakeCuda()) is True
    monkeypatch.setenv("DDIM_COLD_FORCE_REFERENCE", "1")
    assert vit._fused_allowed(_FakeCuda()) is False


def test_lib_path_override():
    r = _py("from ddim_cold_amd.ops import _ext; print(_ext.LIB_PATH); print(_ext.load(False)); print(_ext.error())",
            env={"DDIM_COLD_LIB": "/tmp/other_build/_C.so"})
    assert r.returncode == 0, r.stderr
    out = r.stdout.splitlines()
    assert out[0] == "/tmp/other_build/_C.so" and out[1] == "False" and "/tmp/other_build/_C.so" in out[2]


def test_build_flag_switches():
    code = ("from ddim_cold_amd import build; f = build._flags([], 1); "
            "print(build.ARCH); print('-DX_TEST=1' in f); print('--offload-arch=gfx950' in f)")
    r = _py(code, env={"DDIM_COLD_HIPFLAGS": "-DX_TEST=1"})
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == ["gfx950", "True", "True"]
    r = _py("from ddim_cold_amd import build; print(build.ARCH)", env={"DDIM_COLD_ARCH": "gfx942"})
    assert r.stdout.strip() == "gfx942"
    r = _py("from ddim_cold_amd import build; import inspect; print('DDIM_COLD_ALLOW_SCRATCH' in "
            "inspect.getsource(build._check_scratch))")
    assert r.stdout.strip() == "True"


def test_allow_scratch_warns_instead_of_failing(tmp_path):
    from ddim_cold_amd import build
    log = "remark: foo.hip:1:1: Function Name: k_bad\nremark: foo.hip:1:1:     ScratchSize [bytes/lane]: 16\n"
    with pytest.raises(RuntimeError, match="scratch"):
        build._check_scratch([log])
    os.environ["DDIM_COLD_ALLOW_SCRATCH"] = "1"
    try:
        build._check_scratch([log])
    finally:
        os.environ.pop("DDIM_COLD_ALLOW_SCRATCH")


def test_preissue_switch():
    r = _py("from ddim_cold_amd.train import engine; print(engine.PREISSUE)")
    assert r.stdout.strip() == "True"
    r = _py("from ddim_cold_amd.train import engine; print(engine.PREISSUE)", env={"DDIM_COLD_PREISSUE": "0"})
    assert r.stdout.strip() == "False"


def test_torch_profile_window(tmp_path, monkeypatch):
    from ddim_cold_amd.utils.observe import torch_profiler
    monkeypatch.delenv("DDIM_COLD_TORCH_PROFILE", raising=False)
    assert torch_profiler(0) is None
    monkeypatch.setenv("DDIM_COLD_TORCH_PROFILE", str(tmp_path))
    monkeypatch.setenv("DDIM_COLD_TORCH_PROFILE_STEPS", "1,2")
    prof = torch_profiler(0)
    prof.__enter__()
    for _ in range(4):
        torch.ones(8).sum()
        prof.step()
    prof.__exit__(None, None, None)
    assert os.path.isfile(tmp_path / "trace_rank0.json")


def test_rehearse_shared_gpu_flag_on_cpu():
    """bench.py --gpus 2 with the rehearsal switch: gloo ranks, flagged as not a scaling number."""
    e = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2", DDIM_COLD_REHEARSE_SHARED_GPU="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--no-sampler", "--batch", "4"], capture_output=True, text=True, timeout=600, cwd="/tmp",
                       env=e)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["rehearsal_shared_gpu_gloo"] is True and out["n_gpus"] == 2


def test_bench_deadline_switches_parse():
    """DDIM_COLD_PG_TIMEOUT_S / DDIM_COLD_DEADLINE_S / DDIM_COLD_SPAWN_DEADLINE_S set bench.py's
    process-group timeout and the rank / parent deadlines (the stall tests in
    tests/test_bench_cpu.py exercise the deadlines end to end)."""
    code = "import bench; print(bench.PG_TIMEOUT_S, bench.RANK_DEADLINE_S, bench.SPAWN_DEADLINE_S)"
    r = _py(code)
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == ["120", "450.0", "480.0"]
    r = _py(code, {"DDIM_COLD_PG_TIMEOUT_S": "45", "DDIM_COLD_DEADLINE_S": "100"})
    assert r.stdout.split() == ["45", "100.0", "130.0"]
    r = _py(code, {"DDIM_COLD_SPAWN_DEADLINE_S": "7"})
    assert r.stdout.split()[2] == "7.0"


def test_phase_dir_switch(tmp_path):
    """DDIM_COLD_PHASE_DIR names the directory the ranks' phase markers go to (else one keyed
    by the launcher's run id / master port); report_dir() reads them back."""
    code = ("from ddim_cold_amd.parallel import watchdog as w; print(w.default_dir()); "
            "p = w.PhaseLog(1, 2, echo=False); p.mark('probe'); print(p.dir)")
    r = _py(code, {"DDIM_COLD_PHASE_DIR": str(tmp_path)})
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == [str(tmp_path), str(tmp_path)]
    assert any(f.startswith("rank1") or "1" in f for f in os.listdir(tmp_path))
    r = _py("from ddim_cold_amd.parallel import watchdog as w; print(w.default_dir())", {"MASTER_PORT": "29513"})
    assert r.stdout.strip().endswith("ddim_cold_phases_29513")
