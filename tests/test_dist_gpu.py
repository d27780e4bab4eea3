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
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "dist-parity ok" in r.stdout
