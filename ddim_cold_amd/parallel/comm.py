"""Native RCCL communicator (``csrc/comm.cpp``) for the gradient reducer.

The reference's only hot collective is DDP's bucketed gradient all-reduce
(``multi_gpu_trainer.py:88``, ``:128``) plus the initial parameter broadcast
of the DDP constructor.  ``NativeComm`` is the MI355X-side owner of that
traffic: one ``ncclComm_t`` per process, bootstrapped through the
``torch.distributed`` TCPStore (rank 0 publishes the 128-byte
``ncclUniqueId``), whose collectives go straight onto the caller's current
HIP stream — the train engine's communication stream — so they are captured
into the step hipGraph as plain graph nodes.  ``torch.distributed`` (backend
``nccl`` = RCCL) stays the control plane: rendezvous, barriers, metric
reductions.
"""
from __future__ import annotations

import itertools
import os
from typing import Optional

import torch
import torch.distributed as dist

from ..ops import _ext

_SEQ = itertools.count()

SUM, MAX, MIN = 0, 1, 2


def _store():
    return dist.distributed_c10d._get_default_store()


class ExternalEvent:
    """A HIP event recorded as an external event-record node when captured: the
    capturing graph keeps a single chain (no cross-stream branch), and a stream
    that waits on the event after the graph's replay is enqueued orders after that
    point of the replay (``csrc/comm.cpp`` event_*)."""

    RELEASE_TO_DEVICE = 0x40000000     # hipEventReleaseToDevice
    DISABLE_SYSTEM_FENCE = 0x20000000  # hipEventDisableSystemFence

    def __init__(self, flags: int = 0):
        _ext.load(raise_on_error=True)
        self.handle = int(torch.ops.ddim_cold.event_create(int(flags)))

    def record(self):
        """Record on the current stream (inside a capture: an external node)."""
        torch.ops.ddim_cold.event_record_external(self.handle)

    def wait(self, stream: torch.cuda.Stream):
        with torch.cuda.stream(stream):
            torch.ops.ddim_cold.stream_wait_event(self.handle)

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None:
            try:
                torch.ops.ddim_cold.event_destroy(h)
            except Exception:  # interpreter shutdown
                pass
            self.handle = None


class FlagSignal:
    """Per-bucket hand-off counters for the event-split data-parallel step.

    Inside the compute graph, :meth:`bump` is a 1-lane kernel node that adds 1 to
    ``flags[k]`` with a system-scope release once the bucket's gradients are final;
    the host then orders a comm-stream collective behind ``flags[k] >= replays``
    with a bounded polling kernel (:meth:`waiter`).  Unlike an event-record node,
    the kernel node keeps the graph one uninterrupted chain (measured on MI355X:
    the comm stream waiting on mid-graph event nodes started only after the whole
    graph had finished, so nothing overlapped)."""

    def __init__(self, n: int, device):
        _ext.load(raise_on_error=True)
        self.flags = torch.zeros(max(1, n), dtype=torch.int32, device=device)
        self.err = torch.zeros(1, dtype=torch.int32, device=device)
        self.expected = 0  # replays of the graph that bumps the counters
        # the polling kernel's bound (default 2 s; tests shorten it)
        self.timeout_us = int(os.environ.get("DDIM_COLD_HANDOFF_TIMEOUT_US", "0"))
        # testing: wait for a counter value the compute graph never reaches, so every
        # hand-off times out (exercises the failure path end to end)
        self.skew = int(os.environ.get("DDIM_COLD_TEST_HANDOFF_SKEW", "0"))

    @staticmethod
    def supported(device) -> bool:
        _ext.load(raise_on_error=True)
        d = torch.device(device)
        return bool(torch.ops.ddim_cold.stream_wait_value_supported(d.index if d.index is not None else
                                                                     torch.cuda.current_device()))

    def bump(self, k: int):
        torch.ops.ddim_cold.flag_bump(self.flags, int(k))

    def waiter(self, k: int):
        sig = self

        class _Wait:
            def wait(self_, stream):
                with torch.cuda.stream(stream):  # our bounded 1-lane polling kernel
                    torch.ops.ddim_cold.flag_wait(sig.flags, int(k), int(sig.expected + sig.skew) & 0xFFFFFFFF,
                                                  sig.err, sig.timeout_us)
        return _Wait()

    def failed(self) -> bool:
        return int(self.err.item()) != 0

    def check(self):
        """Raise if a comm-stream wait timed out (its collective then ran on stale data)."""
        if self.failed():
            raise RuntimeError("data-parallel hand-off: a comm-stream flag wait timed out, so a gradient "
                               "bucket was all-reduced before its gradients were final; stopping "
                               "(resume from the last checkpoint; DDIM_COLD_PREISSUE=0 issues the "
                               "collectives after the compute replay)")


class LoopbackPair:
    """Two data-parallel "ranks" in ONE process on ONE device, for testing the
    multi-rank hand-off where RCCL cannot run (it refuses two ranks per device).

    ``endpoint(e)`` is a communicator for engine ``e`` (:meth:`TrainEngine.attach_comm`):
    its ``all_reduce_`` is one launch of ``pair_allreduce_kernel`` (csrc/comm_wire.hip)
    on the caller's stream that waits, on the device, for the OTHER endpoint's
    matching launch and then writes stage[0] + stage[1] -- so engine 0's comm-stream
    work depends on engine 1's compute replay and vice versa, as across real ranks,
    and both replicas get bit-identical sums.  The collective counter lives on the
    device (graph-capturable); waits are bounded (``err``)."""

    def __init__(self, device, max_numel: int, timeout_us: int = 0):
        _ext.load(raise_on_error=True)
        self.device = torch.device(device)
        self.stage = torch.zeros(2, max_numel, dtype=torch.float32, device=self.device)
        self.flags = torch.zeros(int(torch.ops.ddim_cold.pair_flags_size()), dtype=torch.int32, device=self.device)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.timeout_us = int(timeout_us)

    def endpoint(self, e: int) -> "_LoopbackEndpoint":
        return _LoopbackEndpoint(self, int(e))

    def failed(self) -> bool:
        return int(self.err.item()) != 0


class _LoopbackEndpoint:
    def __init__(self, pair: LoopbackPair, e: int):
        self.pair, self.e = pair, e

    def all_reduce_(self, buf: torch.Tensor, op: int = SUM):
        if op != SUM:
            raise NotImplementedError("loopback pair: SUM only")
        p = self.pair
        torch.ops.ddim_cold.pair_all_reduce_(buf, p.stage, p.flags, self.e, p.err, p.timeout_us)

    def info(self):
        return (2, self.e)

    def destroy(self):
        pass


class NativeComm:
    """One RCCL communicator over the ranks of the default process group."""

    def __init__(self, device: torch.device, key: Optional[str] = None, timeout_s: Optional[float] = None):
        """``timeout_s`` bounds ``ncclCommInitRank`` (default
        ``DDIM_COLD_NATIVE_INIT_TIMEOUT_S``, 90 s; 0: unbounded): past it the init raises
        instead of blocking the process forever (csrc/comm.cpp comm_init).  Testing:
        ``DDIM_COLD_TEST_NATIVE_INIT=fail`` raises before the init, ``=hang`` makes the
        init time out."""
        if not dist.is_initialized():
            raise RuntimeError("NativeComm needs an initialised torch.distributed process group (rendezvous)")
        _ext.load(raise_on_error=True)
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("NativeComm is GPU-only (RCCL); use torch.distributed on CPU")
        self.world = dist.get_world_size()
        self.rank = dist.get_rank()
        store = _store()
        key = key or f"ddim_cold/native_comm/{next(_SEQ)}"
        if self.rank == 0:
            uid = torch.ops.ddim_cold.comm_unique_id()
            store.set(key, bytes(uid.tolist()))
        raw = store.get(key)  # blocks until rank 0 has published the id
        uid = torch.tensor(list(raw), dtype=torch.uint8)
        idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
        if timeout_s is None:
            timeout_s = float(os.environ.get("DDIM_COLD_NATIVE_INIT_TIMEOUT_S", "90"))
        hook = os.environ.get("DDIM_COLD_TEST_NATIVE_INIT", "")
        if hook == "fail":
            raise RuntimeError("DDIM_COLD_TEST_NATIVE_INIT=fail: native RCCL communicator init refused (test hook)")
        self.handle = None
        self.handle = int(torch.ops.ddim_cold.comm_init(uid, self.world, self.rank, idx, int(timeout_s * 1000),
                                                        hook == "hang"))
        n, r = torch.ops.ddim_cold.comm_info(self.handle)
        assert (n, r) == (self.world, self.rank), (n, r, self.world, self.rank)

    def all_reduce_(self, buf: torch.Tensor, op: int = SUM):
        torch.ops.ddim_cold.comm_all_reduce_(buf, self.handle, op)

    def all_reduce_many_(self, bufs, op: int = SUM):
        """In-place all-reduces of several buffers as ONE RCCL group (one launch)."""
        torch.ops.ddim_cold.comm_all_reduce_many_(list(bufs), self.handle, op)

    def all_reduce_bf16_wire_(self, buf: torch.Tensor, scratch: torch.Tensor):
        """SUM all-reduce of an fp32 range over a bf16 wire (pack, reduce, unpack)."""
        torch.ops.ddim_cold.comm_all_reduce_bf16_wire_(buf, scratch, self.handle)

    def broadcast_(self, buf: torch.Tensor, root: int = 0):
        torch.ops.ddim_cold.comm_broadcast_(buf, self.handle, root)

    def all_gather_(self, out: torch.Tensor, inp: torch.Tensor):
        """``out`` = every rank's ``inp`` concatenated in rank order (ncclAllGather)."""
        torch.ops.ddim_cold.comm_all_gather_(out, inp, self.handle)

    def info(self):
        """(ranks, my rank) as RCCL reports them (ncclCommCount / ncclCommUserRank)."""
        return tuple(int(v) for v in torch.ops.ddim_cold.comm_info(self.handle))

    def destroy(self):
        if self.handle is not None:
            torch.ops.ddim_cold.comm_destroy(self.handle)
            self.handle = None

    @staticmethod
    def leaked_inits() -> int:
        """Init helper threads left behind by timed-out inits in this process."""
        _ext.load(raise_on_error=True)
        return int(torch.ops.ddim_cold.comm_init_leaked())
