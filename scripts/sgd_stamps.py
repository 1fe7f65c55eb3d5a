"""Per-role block timeline of the fp32 MNIST SGD launch (sgd_finalize_kernel,
lab): eager training steps with per-block [start, end] clock stamps (100 MHz),
then per role the start / end spread relative to the launch's first block.
Roles in grid order: fc1 dW + SGD tiles (196), FC streaming blocks, conv2
Winograd weight blocks (128), conv2 bias (16), conv1 weights + bias (52).
    python scripts/sgd_stamps.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpi_tensorflow_amd import config as C  # noqa: E402
from mpi_tensorflow_amd.ops import native  # noqa: E402
from mpi_tensorflow_amd.runtime.mnist_engine import make_engine  # noqa: E402
from mpi_tensorflow_amd.utils.data import load_mnist_shard  # noqa: E402

B = 64
cfg = C.TrainConfig(batch_size=B, graph=False).validate()
sh = load_mnist_shard(0, 1, synthetic=True, seed=cfg.seed)
eng = make_engine(cfg, sh.train_x, sh.train_y, torch.device("cuda"), 0, 1, None)
k = native().mnist
buf = torch.zeros(2 * 4096, dtype=torch.int64, device="cuda")
eng.train(20)
torch.cuda.synchronize()
k.set_sgd_prof(buf.data_ptr())
try:
    for rep in range(4):
        buf.zero_()
        eng.train(1)
        torch.cuda.synchronize()
        st = buf.cpu().numpy().reshape(-1, 2)
        nb = int((st[:, 1] > 0).sum())
        st = st[:nb]
        rel = (st - st[:, 0].min()) / 100.0  # us
        nfc = nb - 196 - 128 - 16 - 52
        roles = [("fc1 dW+SGD", 196), ("FC stream", nfc), ("conv2 wino", 128),
                 ("conv2 bias", 16), ("conv1", 52)]
        print(f"rep {rep}: {nb} blocks, launch span {rel[:, 1].max():.2f} us")
        o = 0
        for name, n in roles:
            if n <= 0:
                continue
            r = rel[o:o + n]
            dur = r[:, 1] - r[:, 0]
            print(f"  {name:11s} n={n:4d} start {r[:, 0].min():6.2f}-{r[:, 0].max():6.2f}  "
                  f"end {r[:, 1].min():6.2f}-{r[:, 1].max():6.2f}  dur med {np.median(dur):5.2f} "
                  f"max {dur.max():5.2f} us")
            o += n
finally:
    k.set_sgd_prof(0)
