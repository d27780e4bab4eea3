"""Fallback chain of the data-parallel bench on one GPU (1-rank RCCL group through
``bench.py --force-dist``): the first multi-GPU run must finish on a slower path
rather than die, and say so in its JSON line.

* native communicator init refused / hanging (``DDIM_COLD_TEST_NATIVE_INIT``): the
  bench completes on torch.distributed's communicator (ProcessGroupNCCL = RCCL);
* every gradient-exchange layout failing in the autotune
  (``DDIM_COLD_TEST_FAIL_LAYOUTS``): the bench completes on the eager inline
  all-reduce step and reports ``comm_fallback``.

Reference: multi_gpu_trainer.py:25-30 (NCCL process group), :88 (DDP), :212-219.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--force-dist", "--steps", "8", "--warmup", "4", "--no-sampler", "--no-vendor", "--no-gaussian",
        "--no-hires"]


def _bench(env):
    e = dict(os.environ, PYTHONPATH=ROOT)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + ARGS, capture_output=True, text=True,
                       timeout=240, cwd=ROOT, env=e)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0]), r.stderr


@pytest.mark.parametrize("mode", ["fail", "hang"])
def test_bench_completes_on_torch_comm_when_native_init_fails(mode):
    out, err = _bench({"DDIM_COLD_TEST_NATIVE_INIT": mode, "DDIM_COLD_NATIVE_INIT_TIMEOUT_S": "3"})
    c = out["config"]
    assert c["comm"] == "torch", c
    assert c["native_comm_error"] and ("test hook" in c["native_comm_error"] or "timed out" in c["native_comm_error"])
    assert out["value"] > 0 and c["final_loss"] > 0
    assert "phase=native-comm:fallback-torch" in err


def test_bench_completes_on_eager_inline_when_every_layout_fails():
    out, err = _bench({"DDIM_COLD_TEST_FAIL_LAYOUTS": "1"})
    c = out["config"]
    assert c["comm_layout"] == "eager-inline" and c["comm_fallback"], c
    assert c["allreduce"] == "eager-inline-fallback" and c["graph"] is False
    assert c["autotune_dropped"] and all("test hook" in v for v in c["autotune_dropped"].values())
    assert out["value"] > 0 and c["final_loss"] > 0
    assert "phase=comm-fallback:verified" in err


def test_autotune_budget_zero_skips_every_layout_and_falls_back():
    """DDIM_COLD_AUTOTUNE_BUDGET_S=0: the tuning budget is spent before the first candidate,
    every layout is skipped for time, and the bench still completes on the eager inline
    all-reduce."""
    out, err = _bench({"DDIM_COLD_AUTOTUNE_BUDGET_S": "0"})
    c = out["config"]
    assert c["comm_layout"] == "eager-inline" and c["comm_fallback"], c
    assert out["value"] > 0 and c["final_loss"] > 0
