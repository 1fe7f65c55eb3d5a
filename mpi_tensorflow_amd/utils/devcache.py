"""Device-resident copy of a host evaluation set.

The engines evaluate the same test shard many times per run (every
`eval_every` steps; the reference re-feeds it batch by batch on
every step, /root/reference/mpipy.py:86, :169-183), so the images are
uploaded once and kept on the device.  A cached copy is reused only for the
SAME host array object with the same buffer address, shape, strides and
dtype: the cache holds a reference to that object, so its id cannot be
recycled by a temporary (a fresh slice is a new object and always misses).
Labels are never cached - they are small and callers pass placeholder labels
for prediction-only calls (`eval_prediction`).  In-place mutation of a cached
array is not detected: pass a new array instead.
"""

from __future__ import annotations

from typing import Optional

import numpy as np
import torch


def _key(x: np.ndarray):
    return (x.__array_interface__["data"][0], x.shape, x.strides, x.dtype.str)


class DeviceArrayCache:
    def __init__(self):
        self._x: Optional[np.ndarray] = None
        self._key = None
        self._dev: Optional[torch.Tensor] = None

    def get(self, x: np.ndarray, device: torch.device) -> torch.Tensor:
        if self._x is x and self._key == _key(x):
            return self._dev
        dev = torch.from_numpy(np.ascontiguousarray(x, np.float32)).to(device)
        self._x, self._key, self._dev = x, _key(x), dev
        return dev

    def clear(self) -> None:
        self._x = self._key = self._dev = None
