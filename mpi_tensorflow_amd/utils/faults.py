"""Fault injection for the failure-detection tests (failure
detection / fault injection; the reference has neither, it relies on MPI's
default abort-on-error, /root/reference/mpipy.py:195-198).

`MTA_FAULT="RANK:POINT[:MODE][,...]"` makes rank RANK fail when it reaches
the named point: MODE `exit` (default) terminates with exit code FAULT_EXIT
and no cleanup, like a killed process; MODE `hang` blocks forever, like a
rank stuck in a collective (only a watchdog can end it).  Points used by the
trainer and bench.py:

  after_init     - process group initialised, before any communicator
  before_comm    - right before the device communicator is created
  after_comm     - communicator created, before the engine's setup collectives
  before_train   - engine ready, before the first training step

Unset (the default) it costs one dictionary lookup per point.
"""

from __future__ import annotations

import os
import sys
import time

FAULT_EXIT = 99


def _parse(spec: str):
    out = {}
    for item in spec.split(","):
        parts = [p.strip() for p in item.split(":")]
        if len(parts) < 2:
            continue
        try:
            out[(int(parts[0]), parts[1])] = parts[2] if len(parts) > 2 else "exit"
        except ValueError:
            continue
    return out


def maybe_fail(point: str, rank: int) -> None:
    spec = os.environ.get("MTA_FAULT")
    if not spec:
        return
    mode = _parse(spec).get((int(rank), point))
    if mode is None:
        return
    print(f"[rank {rank}] MTA_FAULT: {mode} at {point}", file=sys.stderr, flush=True)
    if mode == "hang":
        while True:
            time.sleep(3600)
    os._exit(FAULT_EXIT)
