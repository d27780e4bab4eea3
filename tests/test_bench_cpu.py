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


def _bench(args, env=None, timeout=600):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py")] + args
    e = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd="/tmp", env=e)


def test_bench_self_spawns_gpus_n_cpu():
    """`python bench.py --gpus 2` without torchrun launches 2 ranks itself (gloo on CPU)."""
    r = _bench(["--gpus", "2", "--steps", "2", "--warmup", "1", "--no-sampler"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert REQUIRED <= set(out)
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["config"]["global_batch"] == 64 and out["config"]["launcher"] == "self-spawn"


def test_bench_world_size_mismatch_fails():
    """Under an env launcher, --gpus must equal the launched world size."""
    r = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-sampler"],
               env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                    "MASTER_PORT": "29599"}, timeout=300)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "WORLD_SIZE=1" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_bench_gaussian_dataset_two_ranks_cpu():
    """--dataset gaussian times the Gaussian DDIM task (sparse time_embed row exchange
    across 2 gloo ranks) and labels the metric / data accordingly (no baseline ratio)."""
    r = _bench(["--gpus", "2", "--steps", "2", "--warmup", "1", "--no-sampler", "--dataset", "gaussian"])
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["metric"].endswith("Gaussian DDIM") and out["vs_baseline"] is None
    assert "Gaussian DDIM" in out["data"] and out["n_gpus"] == 2 and out["value"] > 0


def test_bench_stalled_rank_is_named_before_the_deadline_self_spawn():
    """One rank stalls at the timed phase (the other then waits in the collective
    bracket): `bench.py --gpus 2` exits non-zero well before the driver's 600 s and the
    stderr names the stuck rank and its phase (watchdog phase files + deadlines)."""
    import time
    t0 = time.time()
    r = _bench(["--gpus", "2", "--steps", "2", "--warmup", "1", "--no-sampler"],
               env={"DDIM_COLD_TEST_STALL": "1:timed", "DDIM_COLD_DEADLINE_S": "60",
                    "DDIM_COLD_SPAWN_DEADLINE_S": "75"}, timeout=300)
    dt = time.time() - t0
    assert r.returncode != 0, r.stdout[-2000:]
    assert dt < 150, dt
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    err = r.stderr
    assert "stuck rank(s): rank 1 in phase 'timed'" in err, err[-4000:]
    assert "rank 0: phase 'timed'" in err, err[-4000:]
    # every rank marked its phases on stderr
    assert "phase=pg-ready" in err and "phase=warmup" in err


def test_bench_stalled_rank_torchrun_rank_deadline():
    """Under torchrun (the driver's launcher) each rank's own deadline thread names the
    stuck rank and exits; torchrun then stops the job."""
    import time
    from ddim_cold_amd.parallel.dist import free_port
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps",
           "2", "--warmup", "1", "--no-sampler"]
    t0 = time.time()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd="/tmp",
                       env=dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2", DDIM_COLD_TEST_STALL="0:engine-ready",
                                DDIM_COLD_DEADLINE_S="60"))
    assert r.returncode != 0
    assert time.time() - t0 < 150
    assert "[ddim_cold watchdog]" in r.stderr, r.stderr[-4000:]
    assert "deadline of 60s passed" in r.stderr
    # rank 0 stalled after building its engine; rank 1 went on into the warm-up's collectives
    assert "stuck rank(s): rank 0 in phase 'engine-ready'" in r.stderr, r.stderr[-4000:]
