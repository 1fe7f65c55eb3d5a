"""Step timing: device time from HIP events next to host wall clock.

The reference imports `time` and never uses it (/root/reference/mpipy.py:10,
timer commented out at :78); SURVEY.md §5 asks for per-step device timing
plus host wall clock with eval excluded.  `SegmentTimer` brackets each
training segment (a run of graph replays between eval / sync events) with a
pair of HIP events on the compute stream, so the device time of the segment
is read back without an extra synchronisation; on CPU it degrades to the
host clock.  For kernel-level breakdowns use
`rocprofv3 --kernel-trace --stats -- python mpipy.py ...` (scripts/prof_summary.py
summarises the SQLite output; committed summaries live in profiles/).
"""

from __future__ import annotations

import time
from typing import List, Optional, Tuple

import torch


class SegmentTimer:
    def __init__(self, device: torch.device):
        self.cuda = device.type == "cuda"
        self._open: Optional[Tuple[object, float]] = None
        self._done: List[Tuple[object, object, float, float]] = []
        self.device_ms = 0.0
        self.host_s = 0.0
        self.steps = 0

    def start(self) -> None:
        ev = None
        if self.cuda:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
        self._open = (ev, time.perf_counter())

    def stop(self, steps: int) -> None:
        """Close the open segment; `steps` training steps ran inside it.  The
        caller synchronises the device before reading host time."""
        ev0, t0 = self._open
        ev1 = None
        if self.cuda:
            ev1 = torch.cuda.Event(enable_timing=True)
            ev1.record()
        host = time.perf_counter() - t0
        self._done.append((ev0, ev1, host, steps))
        self._open = None

    def collect(self) -> None:
        """Fold the closed segments (waits for their end events)."""
        for ev0, ev1, host, steps in self._done:
            self.host_s += host
            self.steps += steps
            if self.cuda:
                ev1.synchronize()  # recorded after the segment's last device sync
                self.device_ms += ev0.elapsed_time(ev1)
            else:
                self.device_ms += host * 1e3
        self._done = []

    def step_ms(self) -> float:
        return self.device_ms / max(self.steps, 1)
