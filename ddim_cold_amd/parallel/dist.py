"""Process-group bootstrap and helpers (one process per GPU).

Reference: ``multi_gpu_trainer.py:25-30`` (NCCL over tcp://127.0.0.1:16666,
fixed port, world from the YAML) and ``:212-219`` (mp.Process spawn, no
exit-code checks).  Here:

* backend ``nccl`` (= RCCL on ROCm, rings over xGMI) on GPUs, ``gloo`` on CPU;
* rendezvous from torchrun-style env vars (RANK / WORLD_SIZE / LOCAL_RANK /
  MASTER_ADDR / MASTER_PORT) or explicit arguments; MASTER_ADDR defaults to
  127.0.0.1 and the port is free-picked by the spawner, so several jobs can
  share a host;
* a process-group timeout so a dead rank cannot hang the others forever.
"""
from __future__ import annotations

import datetime
import os
import socket
from typing import Optional

import torch
import torch.distributed as dist


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def env_world():
    return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")), \
        int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0")))


def graph_safe_nccl_env():
    """Environment for RCCL collectives captured in hipGraphs (call before the
    process group exists).  ProcessGroupNCCL's watchdog thread polls the HIP
    events of in-flight eager collectives; with its event cache on, an event of
    a finished eager collective can be recycled into a collective recorded during
    a capture and then polled -- seen on MI355X as the watchdog aborting the
    process ("operation not permitted on an event last recorded in a capturing
    stream").  Each collective then owns its events instead (the captured step
    issues no eager collectives, so nothing is lost)."""
    os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")


def init_distributed(backend: Optional[str] = None, rank: Optional[int] = None, world_size: Optional[int] = None,
                     master_addr: Optional[str] = None, master_port: Optional[int] = None,
                     timeout_s: int = 600) -> bool:
    """Initialise the default process group if world_size > 1. Returns True if distributed."""
    w_env, r_env, _ = env_world()
    world_size = world_size if world_size is not None else w_env
    rank = rank if rank is not None else r_env
    if world_size <= 1:
        return False
    if dist.is_initialized():
        return True
    os.environ.setdefault("MASTER_ADDR", master_addr or "127.0.0.1")
    if master_port is not None:
        os.environ["MASTER_PORT"] = str(master_port)
    os.environ.setdefault("MASTER_PORT", "29511")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    kw = {}
    if backend == "nccl":
        graph_safe_nccl_env()
        local = int(os.environ.get("LOCAL_RANK", rank % max(torch.cuda.device_count(), 1)))
        dev = torch.device("cuda", local)
        torch.cuda.set_device(dev)
        kw["device_id"] = dev
    dist.init_process_group(backend=backend, rank=rank, world_size=world_size,
                            timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return True


def init_single(backend: Optional[str] = None, device_index: int = 0, timeout_s: int = 300) -> bool:
    """A 1-rank process group (RCCL on a GPU, else gloo): exercises the data-parallel
    step (comm stream, collectives, hand-offs) on one device.  Returns True."""
    if dist.is_initialized():
        return True
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    own_port = "MASTER_PORT" not in os.environ
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    kw = {}
    if backend == "nccl":
        graph_safe_nccl_env()
        torch.cuda.set_device(device_index)
        kw["device_id"] = torch.device("cuda", device_index)
    # a port found free can be taken before the store binds it (other processes' RCCL
    # bootstrap sockets are ephemeral too: seen once as EADDRINUSE in the GPU suite) --
    # a port we picked ourselves is re-picked
    for attempt in range(5):
        if own_port:
            os.environ["MASTER_PORT"] = str(free_port())
        try:
            dist.init_process_group(backend, rank=0, world_size=1, timeout=datetime.timedelta(seconds=timeout_s),
                                    **kw)
            return True
        except Exception as e:  # torch.distributed.DistNetworkError
            if not own_port or attempt == 4 or "EADDRINUSE" not in str(e) and "address already in use" not in str(e):
                raise
    return True


def is_main() -> bool:
    return not dist.is_initialized() or dist.get_rank() == 0


def world_size() -> int:
    return dist.get_world_size() if dist.is_initialized() else 1


def rank() -> int:
    return dist.get_rank() if dist.is_initialized() else 0


def barrier():
    if dist.is_initialized():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def all_reduce_max(x: float, device) -> float:
    if not dist.is_initialized():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_reduce_mean(x: float, device) -> float:
    """Reference metric reduction (multi_gpu_trainer.py:143-145): SUM then / world."""
    if not dist.is_initialized():
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item()) / dist.get_world_size()


def cleanup():
    if dist.is_initialized():
        dist.destroy_process_group()
