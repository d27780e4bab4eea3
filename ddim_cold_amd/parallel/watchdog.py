"""Per-rank phase markers and a wall-clock deadline for multi-process runs.

The reference launches one process per GPU and joins them without looking at
exit codes (``multi_gpu_trainer.py:212-219``); a rank stuck in NCCL init or in a
collective hangs the job silently until something outside kills it.  Here every
rank records the boundary it last crossed -- process-group init, native RCCL
init (+ verified ranks), the all-reduce probe, each autotune layout, capture,
warm-up, timed steps -- as

* one flushed line on stderr (``[ddim_cold] rank 3/8 +12.4s phase=autotune:overlap-2``), and
* a small JSON file per rank in a shared directory (``DDIM_COLD_PHASE_DIR``, or a
  per-job directory under ``/tmp`` keyed by the launcher's run id / master port),
  which the deadline handlers read to name every rank's last phase.

Two deadlines, both well inside an outer job timeout:

* :meth:`PhaseLog.start_deadline` -- a daemon thread in every rank; when the
  deadline passes it prints the report of ALL ranks' last phases (ranks behind
  the others are named as stuck) and ends the process with ``os._exit`` (the
  main thread may be blocked in a C++ collective; torchrun then stops the rest);
* :func:`report_dir` -- used by the self-spawning parent (``bench.py
  spawn_ranks``) to name each rank's last phase when it terminates the children.

Testing hook: ``DDIM_COLD_TEST_STALL=<rank>:<phase>`` makes that rank sleep when
it marks that phase (a rank that never reaches the next collective).
"""
from __future__ import annotations

import json
import os
import sys
import threading
import time
from typing import Dict, Optional

_T0 = time.time()  # process start (module import) for the default deadline
_LOG: Optional["PhaseLog"] = None


def default_dir() -> str:
    """Phase directory shared by the ranks of one job (same value on every rank)."""
    d = os.environ.get("DDIM_COLD_PHASE_DIR")
    if d:
        return d
    key = os.environ.get("TORCHELASTIC_RUN_ID") or os.environ.get("MASTER_PORT") or str(os.getppid())
    key = "".join(ch if ch.isalnum() or ch in "-_" else "_" for ch in key)
    return os.path.join("/tmp", f"ddim_cold_phases_{key}")


class PhaseLog:
    def __init__(self, rank: int, world: int, directory: Optional[str] = None, echo: bool = True,
                 stream=None):
        self.rank, self.world = int(rank), int(world)
        self.dir = directory or default_dir()
        self.echo = echo
        self.stream = stream if stream is not None else sys.stderr
        self.seq = 0
        self.phase = "start"
        self.t_phase = time.time()
        self._lock = threading.Lock()
        self._deadline_thread = None
        self.fired = False
        try:
            os.makedirs(self.dir, exist_ok=True)
        except OSError:
            self.dir = None
        stall = os.environ.get("DDIM_COLD_TEST_STALL", "")
        self._stall = None
        if ":" in stall:
            r, ph = stall.split(":", 1)
            if r.strip().isdigit() and int(r) == self.rank:
                self._stall = ph.strip()

    # ------------------------------------------------------------------ marks
    def mark(self, phase: str, **info):
        with self._lock:
            self.seq += 1
            self.phase = phase
            self.t_phase = time.time()
            self._rec = {"rank": self.rank, "world": self.world, "seq": self.seq, "phase": phase, "t": self.t_phase,
                         "pid": os.getpid(), "info": {k: _jsonable(v) for k, v in info.items()}}
            self._write()
        if self.echo:
            extra = "".join(f" {k}={_short(v)}" for k, v in info.items())
            print(f"[ddim_cold] rank {self.rank}/{self.world} +{self.t_phase - _T0:.1f}s phase={phase}{extra}",
                  file=self.stream, flush=True)
        if self._stall is not None and phase == self._stall:
            print(f"[ddim_cold] rank {self.rank}: DDIM_COLD_TEST_STALL -> stalling in phase {phase}",
                  file=self.stream, flush=True)
            while True:  # a rank that never reaches the next collective
                time.sleep(3600)

    def _write(self):
        if self.dir is None:
            return
        path = os.path.join(self.dir, f"rank{self.rank}.json")
        tmp = path + f".{os.getpid()}.tmp"
        try:
            with open(tmp, "w") as f:
                json.dump(self._rec, f)
            os.replace(tmp, path)
        except OSError:
            pass

    def heartbeat(self):
        """Add where the main thread is now (innermost Python frames, and whether it is
        blocked in a collective / device synchronize) to this rank's phase record."""
        where, waiting = main_thread_where()
        with self._lock:
            rec = getattr(self, "_rec", None)
            if rec is None:
                return
            rec["where"], rec["waiting"], rec["t_beat"] = where, waiting, time.time()
            self._write()

    def report(self) -> str:
        if not self.dir:
            return f"rank {self.rank}: last phase {self.phase}"
        # records older than this job (a reused directory) are ignored
        return report_dir(self.dir, self.world, since=_T0 - 120.0)

    # ------------------------------------------------------------------ deadline
    def start_deadline(self, seconds: float, exit_code: int = 124, since: Optional[float] = None):
        """Daemon thread: once ``seconds`` have passed since ``since`` (default: process
        start), print this rank's phase and every rank's last phase, then ``os._exit``."""
        t_end = (since if since is not None else _T0) + float(seconds)

        def run():
            beat = 0.0
            while True:
                left = t_end - time.time()
                if left <= 0:
                    break
                if time.time() - beat >= HEARTBEAT_S:
                    beat = time.time()
                    self.heartbeat()
                time.sleep(min(left, 1.0))
            self.fired = True
            self.heartbeat()
            time.sleep(1.5)  # the other ranks' deadline threads record where they are too
            msg = (f"[ddim_cold watchdog] rank {self.rank}/{self.world}: deadline of {seconds:.0f}s passed "
                   f"in phase '{self.phase}' (entered {time.time() - self.t_phase:.1f}s ago); stopping.\n"
                   f"{self.report()}")
            try:
                print(msg, file=self.stream, flush=True)
            finally:
                os._exit(exit_code)
        th = threading.Thread(target=run, name="ddim_cold_deadline", daemon=True)
        th.start()
        self._deadline_thread = th
        return th


def report_dir(directory: str, world: int, since: float = 0.0) -> str:
    """One line per rank with its last phase and how long ago it entered it; ranks
    whose phase sequence is behind the furthest rank are named as stuck.  Records
    written before ``since`` (an earlier job in the same directory) are ignored."""
    recs: Dict[int, dict] = {}
    for r in range(int(world)):
        try:
            with open(os.path.join(directory, f"rank{r}.json")) as f:
                v = json.load(f)
            if float(v.get("t", 0.0)) >= since:
                recs[r] = v
        except (OSError, ValueError):
            pass
    now = time.time()
    lines = []
    top = max((v["seq"] for v in recs.values()), default=0)
    behind = [r for r in range(world) if r not in recs or recs[r]["seq"] < top]
    if not behind:
        # every rank reached the same boundary: the ones NOT blocked in a collective /
        # device synchronize are holding up the ones that are
        waiting = {r for r, v in recs.items() if v.get("waiting")}
        if waiting and len(waiting) < len(recs):
            behind = [r for r in recs if r not in waiting]
    behind = sorted(behind)
    for r in range(int(world)):
        v = recs.get(r)
        if v is None:
            lines.append(f"  rank {r}: no phase recorded (never started, or died before the first marker)")
            continue
        tag = "  <- behind (stuck here)" if r in behind else ""
        info = "".join(f" {k}={_short(x)}" for k, x in v.get("info", {}).items())
        where = ""
        if v.get("where"):
            where = f"\n      {'waiting in a collective' if v.get('waiting') else 'running'} at {v['where']}"
        lines.append(f"  rank {r}: phase '{v['phase']}' (#{v['seq']}) for {now - v['t']:.1f}s{info}{tag}{where}")
    if behind:
        head = "stuck rank(s): " + ", ".join(
            f"rank {r} in phase '{recs[r]['phase']}'" if r in recs else f"rank {r} (no phase)" for r in behind)
    elif recs:
        ph = {v["phase"] for v in recs.values()}
        head = f"all ranks stuck in the same phase: {', '.join(sorted(ph))} (a collective that never completes)"
    else:
        head = "no rank recorded a phase"
    return f"[ddim_cold watchdog] {head}\n" + "\n".join(lines)


HEARTBEAT_S = 5.0
# innermost frames that mean "blocked on other ranks / the device", not "stuck here"
_WAIT_FILES = (os.sep + "distributed" + os.sep,)
_WAIT_FUNCS = {"synchronize", "barrier", "all_reduce", "all_gather", "all_gather_into_tensor", "broadcast",
               "all_reduce_max", "all_reduce_mean", "wait", "get", "item"}


def main_thread_where(depth: int = 3):
    """(``"file:line func <- ..."`` of the main thread's innermost frames, blocked?)."""
    import threading as _th
    fr = sys._current_frames().get(_th.main_thread().ident)
    parts, waiting = [], False
    k = 0
    while fr is not None and k < 12:
        co = fr.f_code
        if k < depth:
            parts.append(f"{os.path.basename(co.co_filename)}:{fr.f_lineno} {co.co_name}")
        if k < 4 and (co.co_name in _WAIT_FUNCS or any(w in co.co_filename for w in _WAIT_FILES)):
            waiting = True
        fr = fr.f_back
        k += 1
    return " <- ".join(parts), waiting


def _jsonable(v):
    if isinstance(v, (int, float, str, bool)) or v is None:
        return v
    return str(v)


def _short(v) -> str:
    s = str(v)
    return s if len(s) <= 80 else s[:77] + "..."


# ---------------------------------------------------------------------- module-level log
def install(rank: int, world: int, directory: Optional[str] = None, deadline_s: Optional[float] = None,
            echo: bool = True, since: Optional[float] = None) -> PhaseLog:
    """Create the process's phase log (and its deadline thread if ``deadline_s``,
    counted from ``since``: default the import of this module; pass the process's
    start time to include the interpreter / torch import)."""
    global _LOG, _T0
    if since is not None:
        _T0 = float(since)
    _LOG = PhaseLog(rank, world, directory, echo=echo)
    _LOG.mark("start", pid=os.getpid())
    if deadline_s is not None and deadline_s > 0:
        _LOG.start_deadline(deadline_s)
    return _LOG


def phase(name: str, **info):
    """Record a phase boundary (no-op unless :func:`install` ran in this process)."""
    if _LOG is not None:
        _LOG.mark(name, **info)


def current() -> Optional[PhaseLog]:
    return _LOG
