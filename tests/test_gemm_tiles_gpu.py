"""Every GEMM tile configuration (32x64, 64x64, 128x64, 128x128) against the fp32 references:
re-runs the GEMM tests of test_kernels_gpu.py in a child process per forced tile choice
(the choice is read once per process from DDIM_COLD_GEMM_TILE)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.parametrize("tile", [0, 1, 2, 3])
def test_gemm_tile_configs(tile):
    env = dict(os.environ, DDIM_COLD_GEMM_TILE=str(tile), PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_kernels_gpu.py"), "-k",
                        "linear or qkv or resid or gelu or dgrad or head or patch"],
                       capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
