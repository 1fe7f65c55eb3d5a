"""Learning-rate schedule of the reference.

`tf.train.exponential_decay(0.01, iter_ * batch_size, train_data.shape[0],
0.95, staircase=True)` (`/root/reference/mpipy.py:59-64`):

    lr(step) = 0.01 * 0.95 ** floor(step * 64 / N_local)

where `iter_` is the float32 global step read BEFORE the optimizer
increments it (`minimize(global_step=iter_)`, `:65-66`), so step s trains
with lr(s).  N_local is the per-rank train-buffer row count, which makes
the decay happen once per LOCAL epoch (quirk Q15 kept on purpose).

The HIP SGD kernel evaluates the same formula in fp32 on the device from
the device-side step counter (`csrc/kernels/sgd.hip`).
"""

from __future__ import annotations

import numpy as np

from ..config import BASE_LR, BATCH_SIZE, LR_DECAY


def decay_exponent(step: int, n_local: int, batch: int = BATCH_SIZE) -> int:
    return (step * batch) // n_local


def learning_rate(step: int, n_local: int, batch: int = BATCH_SIZE, base: float = BASE_LR,
                  decay: float = LR_DECAY) -> float:
    """fp32 value identical to what the device computes."""
    e = np.float32(decay_exponent(step, n_local, batch))
    return float(np.float32(base) * np.power(np.float32(decay), e, dtype=np.float32))
