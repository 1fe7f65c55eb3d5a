"""Counter-based dropout RNG shared bit-for-bit by the HIP kernels and the
PyTorch oracle.

The reference draws its dropout mask with TF1's stateful Philox stream
(`tf.nn.dropout(hidden, 0.5, seed=1)`, `/root/reference/mpipy.py:166`); that
stream cannot be reproduced outside TF, and its op seed is identical on every
rank (quirk Q14).  Here each mask element is a pure function of
(seed, rank, step, element index), so it needs no RNG state on the device
(graph-capturable: the step comes from the device-side step counter) and
the oracle can regenerate exactly the mask a kernel used.

    key  = mix(mix(seed * 0x9E3779B9 + rank) ^ (step * 0x85EBCA6B + salt))
    u    = (mix(index ^ key) >> 8) * 2^-24          in [0, 1)
    keep = u < keep_prob,  scale = 1 / keep_prob

`mix` is a 32-bit integer avalanche hash (xor-shift / multiply).  The HIP
side lives in `csrc/kernels/common.h` (`dropout_key`, `dropout_keep`).
"""

from __future__ import annotations

import numpy as np

M32 = 0xFFFFFFFF
GOLDEN = 0x9E3779B9
STEP_MUL = 0x85EBCA6B
EVAL_SALT = 0x5BD1E995  # separates the eval-time (quirk Q8) stream


def _mix_np(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64) & M32
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & M32
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & M32
    x ^= x >> np.uint64(16)
    return x


def dropout_key(seed: int, rank: int, step: int, salt: int = 0) -> int:
    a = _mix_np(np.array([(seed * GOLDEN + rank) & M32], np.uint64))[0]
    b = np.uint64(((step * STEP_MUL) + salt) & M32)
    return int(_mix_np(np.array([a ^ b], np.uint64))[0])


def keep_mask_np(key: int, n: int, keep_prob: float) -> np.ndarray:
    idx = np.arange(n, dtype=np.uint64)
    h = _mix_np(idx ^ np.uint64(key))
    u = (h >> np.uint64(8)).astype(np.float64) * (2.0 ** -24)
    return u < np.float32(keep_prob)


def keep_mask_torch(key: int, shape, keep_prob: float, device=None):
    """Same mask as a torch bool tensor (computed with numpy on the host)."""
    import torch

    n = 1
    for s in shape:
        n *= int(s)
    m = keep_mask_np(key, n, keep_prob).reshape(tuple(shape))
    return torch.from_numpy(m).to(device=device)
