"""Observability / debugging aids of the trainer.

* :class:`StepClock` — device-side (HIP event) timing of log windows: no host
  synchronisation inside the step loop, read only at log points.
* :func:`range_push` / :func:`range_pop` — roctx ranges (through
  ``torch.cuda.nvtx``, which ROCm builds route to roctx) around trainer phases,
  visible in ``rocprofv3 --marker-trace``; no-ops where unavailable.
* :func:`torch_profiler` — optional ``torch.profiler`` capture of a step window
  (``DDIM_COLD_TORCH_PROFILE=<dir>``, ``DDIM_COLD_TORCH_PROFILE_STEPS=a,b``).
* :func:`check_param_sync` — cross-rank parameter checksum (debug mode
  ``sync_check_every``): raises if data-parallel replicas diverged.
* :class:`FaultInjected` — raised by ``fault_inject_step`` to test resume.
"""
from __future__ import annotations

import contextlib
import os
from typing import Optional

import torch
import torch.distributed as dist


class FaultInjected(RuntimeError):
    pass


class StepClock:
    """HIP-event clock over log windows (falls back to host time on CPU)."""

    def __init__(self, device: torch.device):
        self.cuda = torch.device(device).type == "cuda"
        self.last = None
        self.last_steps = 0
        if not self.cuda:
            import time
            self._now = time.perf_counter

    def mark(self, steps: int):
        """Returns (seconds, steps) since the previous mark (None on the first call)."""
        if self.cuda:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            ev.synchronize()
            out = None
            if self.last is not None:
                out = (self.last.elapsed_time(ev) / 1e3, steps - self.last_steps)
            self.last, self.last_steps = ev, steps
            return out
        now = self._now()
        out = None if self.last is None else (now - self.last, steps - self.last_steps)
        self.last, self.last_steps = now, steps
        return out


def range_push(name: str):
    try:
        torch.cuda.nvtx.range_push(name)
    except Exception:
        pass


def range_pop():
    try:
        torch.cuda.nvtx.range_pop()
    except Exception:
        pass


@contextlib.contextmanager
def phase(name: str):
    range_push(name)
    try:
        yield
    finally:
        range_pop()


def torch_profiler(rank: int):
    """A ``torch.profiler.profile`` (entered by the caller) when DDIM_COLD_TORCH_PROFILE is set, else None."""
    out = os.environ.get("DDIM_COLD_TORCH_PROFILE")
    if not out:
        return None
    a, b = (int(v) for v in os.environ.get("DDIM_COLD_TORCH_PROFILE_STEPS", "10,15").split(","))
    from torch.profiler import ProfilerActivity, profile, schedule
    acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if torch.cuda.is_available() else [])
    os.makedirs(out, exist_ok=True)

    def handler(p):
        p.export_chrome_trace(os.path.join(out, f"trace_rank{rank}.json"))

    return profile(activities=acts, schedule=schedule(wait=a, warmup=0, active=max(1, b - a), repeat=1),
                   on_trace_ready=handler)


def param_checksum(flat: torch.Tensor) -> torch.Tensor:
    f = flat.double()
    return torch.stack([f.sum(), (f * f).sum(), f.abs().max()])


def check_param_sync(flat: torch.Tensor, group=None, step: Optional[int] = None, rtol: float = 0.0):
    """All ranks must hold identical parameters: compare checksums via MAX / MIN all-reduce."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return
    cs = param_checksum(flat)
    hi, lo = cs.clone(), cs.clone()
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    if not torch.all((hi - lo).abs() <= rtol * hi.abs()):
        raise RuntimeError(f"data-parallel replicas diverged at step {step}: checksum max {hi.tolist()} "
                           f"min {lo.tolist()}")


@contextlib.contextmanager
def no_gc():
    """Collect, then keep Python's cyclic GC off for the block (hipGraph stream
    capture): a collection during capture can run destructors of an earlier,
    unreferenced graph or of tensors tied to another stream -- HIP calls that
    are illegal while a stream is being captured (seen as an abort inside a
    captured op)."""
    import gc
    gc.collect()
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


def drain_before_capture(device) -> None:
    """Quiesce before a hipGraph capture that follows eager collectives.

    1. ``synchronize``: every eager kernel and collective of this rank has finished.
    2. With a process group: a barrier, so every rank has too (no peer is still
       inside a collective this rank's capture would wait behind).
    3. One watchdog period (ProcessGroupNCCL polls its pending work every ~100 ms):
       the finished works are then dropped instead of being queried while the
       capture is open.  The capture itself is thread-local (``CAPTURE_MODE``), so a
       late watchdog query can no longer invalidate it -- the wait only keeps the
       watchdog's event queries and the capture apart, it is not what makes the
       capture correct.
    """
    import time
    from ..parallel.dist import barrier
    if device is not None and torch.device(device).type == "cuda":
        torch.cuda.synchronize(device)
    if dist.is_available() and dist.is_initialized():
        barrier()
        if device is not None and torch.device(device).type == "cuda":
            torch.cuda.synchronize(device)
        time.sleep(0.15)


def is_capture_error(e: BaseException) -> bool:
    """A failure of the graph capture itself (an op illegal during capture, an
    invalidated capture) -- as opposed to an error in the captured work.  Matched
    on the HIP runtime's capture error names / messages (and torch's own capture
    checks), not on any message that merely mentions a graph."""
    if not isinstance(e, RuntimeError):
        return False
    msg = str(e)
    return any(s in msg for s in CAPTURE_ERROR_MARKERS)


# HIP error names a failed stream capture surfaces as (hipGetErrorName) and the
# runtime's hipGetErrorString texts for them -- torch reports the latter (the strings
# are the ones libamdhip64.so of ROCm 7.2 carries) -- plus torch's own "not allowed
# while capturing" checks
CAPTURE_ERROR_MARKERS = (
    "hipErrorStreamCaptureUnsupported", "hipErrorStreamCaptureInvalidated", "hipErrorStreamCaptureMerge",
    "hipErrorStreamCaptureUnmatched", "hipErrorStreamCaptureUnjoined", "hipErrorStreamCaptureIsolation",
    "hipErrorStreamCaptureImplicit", "hipErrorStreamCaptureWrongThread", "hipErrorCapturedEvent",
    "operation not permitted when stream is capturing",
    "operation failed due to a previous error during capture",
    "operation would result in a merge of separate capture sequences",
    "capture was not ended in the same stream as it began",
    "capturing stream has unjoined work",
    "dependency created on uncaptured work in another stream",
    "operation would make the legacy stream depend on a capturing blocking stream",
    "operation not permitted on an event last recorded in a capturing stream",
    "attempt to terminate a thread-local capture sequence from another thread",
    "capture sequence", "stream is capturing", "during CUDA graph capture", "during graph capture",
)
