"""Collective watchdog: turns a dead peer or a hung collective into a prompt,
non-zero exit of every rank instead of a hang.

The reference has no failure handling beyond one broken `try/except`
(`/root/reference/mpipy.py:195-198`); it relies on MPI's default error
handler, which aborts the whole job when a rank dies.  On MI355X the
gradient all-reduces are RCCL kernels replayed inside hipGraphs, and a
collective whose peer died simply never completes: the host blocks forever
in the next device synchronize.  This watchdog restores MPI's "abort the
job" semantics:

* a daemon thread polls `ncclCommGetAsyncError` on every registered
  communicator (any non-success, non-in-progress code is fatal);
* training code arms a deadline around every region that waits on the
  device (`with wd.guard("train steps 100..124"):`); if the region has not
  finished `timeout_s` after it was armed, the rank is declared hung;
* on either failure the thread `ncclCommAbort`s every communicator (which
  makes in-flight RCCL kernels exit, so the GPU drains), prints the rank,
  the region and the reason on stderr and terminates the process with
  `EXIT_CODE` via `os._exit` (no re-exec; the launcher - torchrun / mpirun /
  bench.py's own spawner - then tears down the remaining ranks).

Communicators are any objects with `async_error() -> int` and `abort()`
(the native `_C.RcclComm` and `_C.ShmComm`, or a fake in the CPU tests);
others are ignored and only the deadline applies (gloo, emulated and
host-staged comms).  The watchdog exists BEFORE the communicators: start-up
(communicator creation, the engines' connection-setup collectives) runs
under a deadline too, and communicators are registered with `add()` as they
appear.

The deadline is a heartbeat, not a budget for a whole run: `run_in_chunks`
splits a long run of training steps into chunks, each armed on its own and
sized from the measured step time to a fraction of the deadline, so a slow
but progressing run is never declared hung.
"""

from __future__ import annotations

import contextlib
import os
import sys
import threading
import time
from typing import Callable, Iterable, List, Optional

EXIT_CODE = 70  # EX_SOFTWARE
NCCL_SUCCESS = 0
NCCL_IN_PROGRESS = 7


class CollectiveWatchdog:
    def __init__(self, comms: Iterable = (), timeout_s: float = 600.0, rank: int = 0,
                 poll_s: float = 0.05, exit_fn: Optional[Callable[[int], None]] = None,
                 describe_error: Optional[Callable[[int], str]] = None):
        self.comms: List = [c for c in comms
                            if c is not None and hasattr(c, "async_error") and hasattr(c, "abort")]
        self.timeout_s = float(timeout_s)
        self.rank = rank
        self.poll_s = poll_s
        self._exit = exit_fn or os._exit
        self._describe = describe_error
        self._lock = threading.Lock()
        self._deadline: Optional[float] = None
        self._what = ""
        self._stop = threading.Event()
        self.fired: Optional[str] = None
        self._thread = threading.Thread(target=self._run, name="collective-watchdog", daemon=True)
        self._thread.start()

    def add(self, comm) -> None:
        """Registers a communicator created after the watchdog (DeviceComm
        wrappers are unwrapped to their native handle)."""
        if comm is None:
            return
        h = getattr(comm, "native_handle", None)
        c = h if h is not None else comm
        if hasattr(c, "async_error") and hasattr(c, "abort"):
            with self._lock:
                if all(c is not o for o in self.comms):
                    self.comms.append(c)

    # ---------------------------------------------------------------- arming
    def arm(self, what: str, timeout_s: Optional[float] = None) -> None:
        with self._lock:
            self._what = what
            self._deadline = time.monotonic() + (self.timeout_s if timeout_s is None else timeout_s)

    def disarm(self) -> None:
        with self._lock:
            self._deadline = None

    @contextlib.contextmanager
    def guard(self, what: str, timeout_s: Optional[float] = None):
        """Arms the deadline for the body (typically: launch work + device
        synchronize); the body must end with the device drained."""
        self.arm(what, timeout_s)
        try:
            yield self
        finally:
            self.disarm()

    def stop(self) -> None:
        self._stop.set()
        self._thread.join(timeout=2.0)

    # ---------------------------------------------------------------- thread
    def _check_async(self) -> Optional[str]:
        with self._lock:
            comms = list(self.comms)
        for c in comms:
            try:
                e = int(c.async_error())
            except Exception as ex:  # a broken communicator is itself fatal
                return f"async-error query failed ({ex})"
            if e not in (NCCL_SUCCESS, NCCL_IN_PROGRESS):
                if hasattr(c, "error_message"):  # shared-memory communicator
                    msg = c.error_message()
                else:
                    msg = self._describe(e) if self._describe else ""
                return f"RCCL asynchronous error {e}{' (' + msg + ')' if msg else ''}"
        return None

    def _run(self) -> None:
        while not self._stop.wait(self.poll_s):
            reason = self._check_async()
            with self._lock:
                dl, what = self._deadline, self._what
            if reason is None and dl is not None and time.monotonic() > dl:
                reason = f"collective deadline of {self.timeout_s:g} s exceeded"
            if reason is not None:
                self._fail(reason, what if dl is not None else "idle")
                return

    def _fail(self, reason: str, what: str) -> None:
        self.fired = reason
        print(f"[rank {self.rank}] collective watchdog: {reason} during {what}; "
              f"aborting {len(self.comms)} communicator(s) and exiting with {EXIT_CODE}",
              file=sys.stderr, flush=True)
        with self._lock:
            comms = list(self.comms)
        for c in comms:
            try:
                c.abort()
            except Exception:
                pass
        sys.stdout.flush()
        self._exit(EXIT_CODE)


_NULL = contextlib.nullcontext()


class NullWatchdog:
    """Single-rank runs: nothing to watch."""

    comms: List = []
    fired = None
    timeout_s = float("inf")

    def add(self, comm):
        pass

    def arm(self, what, timeout_s=None):
        pass

    def disarm(self):
        pass

    def guard(self, what, timeout_s=None):
        return _NULL

    def stop(self):
        pass


def run_in_chunks(wd, train: Callable[[int], None], sync: Callable[[], None], k: int,
                  label: str, first_step: int = 0, granule: int = 1,
                  state: Optional[dict] = None) -> None:
    """Runs train(k) as consecutive train(n) + sync() chunks, each guarded by
    its own deadline (a heartbeat).  The chunk length is a multiple of
    `granule` (the engine's captured-graph length) sized so a chunk takes
    about a quarter of the deadline at the step time measured so far
    (`state["step_s"]`, carried across calls).  A hang is still caught
    within one deadline; a long healthy run is never mistaken for one."""
    st = state if state is not None else {}
    g = max(1, int(granule))
    budget = getattr(wd, "timeout_s", float("inf"))
    done = 0
    while done < k:
        step_s = st.get("step_s")
        if budget == float("inf"):  # nothing watches: one chunk
            n = k - done
        elif step_s is None:  # first chunk measures the step time
            n = g
        else:
            n = max(g, int(0.25 * budget / max(step_s, 1e-9)) // g * g)
        n = min(n, k - done)
        s0 = first_step + done
        t0 = time.monotonic()
        with wd.guard(f"{label} {s0}..{s0 + n - 1}"):
            train(n)
            sync()
        st["step_s"] = (time.monotonic() - t0) / n
        done += n


def make_watchdog(comms: Iterable, timeout_s: float, rank: int, world: int):
    """A CollectiveWatchdog when there is something to watch (world > 1),
    otherwise a no-op.  `comms` may hold DeviceComm wrappers or raw native
    communicators; wrappers are unwrapped to their native handle."""
    if world <= 1:
        return NullWatchdog()
    raw = []
    for c in comms:
        if c is None:
            continue
        h = getattr(c, "native_handle", None)
        raw.append(h if h is not None else c)
    describe = None
    try:
        from ..ops import native

        C = native()
        describe = C.RcclComm.error_string if C.RcclComm.loaded() else None
    except Exception:
        pass
    return CollectiveWatchdog(raw, timeout_s, rank, describe_error=describe)
