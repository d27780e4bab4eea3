"""bench.py contract on CPU: torchrun, 2 gloo ranks, one JSON line from rank 0 with the
required keys (the driver launches exactly this command shape with N GPUs)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config"}


def test_bench_torchrun_two_ranks_cpu():
    from ddim_cold_amd.parallel.dist import free_port
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps",
           "2", "--warmup", "1", "--no-sampler"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd="/tmp",
                       env=dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2"))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert REQUIRED <= set(out)
    assert out["n_gpus"] == 2 and out["steps"] == 2 and out["warmup"] == 1
    assert out["config"]["global_batch"] == 64 and out["config"]["parallelism"] == "dp2"
    assert out["higher_is_better"] is True and out["scaling"] == "weak" and out["value"] > 0
