"""Distributed engine paths on one GPU (1-rank RCCL group, run in a child process so the
test process keeps no process group): captured and segmented collectives reproduce the
single-process step bit for bit."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_rccl_engine_paths_match_single_process():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "dist_parity.py")], capture_output=True,
                       text=True, timeout=600, env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0, "\n".join(l for l in (r.stdout + r.stderr).splitlines()
                                        if not l.startswith("[W") and "amdgpu.ids" not in l)[-3000:]
    assert "dist-parity ok" in r.stdout


@pytest.mark.gpu
def test_two_ranks_one_gpu_gloo_match_single_process():
    """Two data-parallel ranks on one GPU over gloo (RCCL allows one rank per device):
    real cross-rank gradient traffic through the event-split step and autotune_comm()."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "dist2_gpu.py")], capture_output=True,
                       text=True, timeout=600, env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0, "\n".join(l for l in (r.stdout + r.stderr).splitlines()
                                        if not l.startswith("[W") and "amdgpu.ids" not in l)[-3000:]
    assert "dist2-gpu ok" in r.stdout
