"""Log lines (reference-exact formats) and JSONL metrics.

Reference output (`/root/reference/mpipy.py:77`, `:88`, `:90`):

    print("Process ID:", rank, " training session starts!")
        -> "Process ID: 0  training session starts!"
    print(rank, ' process at ', step, 'with test error: %.1f%%' % err)
        -> "0  process at  50 with test error: 3.2%"
    sys.stdout.flush()

The same strings are produced here (Python 3 print with default sep), plus
an optional JSON-lines metrics file carrying loss, lr, throughput, timings.
"""

from __future__ import annotations

import json
import sys
import time
from typing import Optional


def start_line(rank: int) -> str:
    return " ".join(["Process ID:", str(rank), " training session starts!"])


def progress_line(rank: int, step: int, test_error: float) -> str:
    return " ".join([str(rank), " process at ", str(step), "with test error: %.1f%%" % test_error])


def emit(line: str, quiet: bool = False) -> None:
    if not quiet:
        print(line)
        sys.stdout.flush()


class MetricsWriter:
    def __init__(self, path: Optional[str], rank: int):
        self.f = open(path, "a") if (path and rank == 0) else None
        self.rank = rank

    def write(self, **kw) -> None:
        if self.f is None:
            return
        kw.setdefault("time", time.time())
        self.f.write(json.dumps(kw, sort_keys=True) + "\n")
        self.f.flush()

    def close(self) -> None:
        if self.f is not None:
            self.f.close()
            self.f = None
