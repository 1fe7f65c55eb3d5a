"""Per-role block timeline of the fp32 merged conv2 backward launch
(conv2_bwd_wino_kernel, lab): eager training steps with per-block clock
stamps (100 MHz); per role the start / end spread relative to the launch's
first block start, and the per-CU-slot chains.
    python scripts/c2bw_stamps.py"""
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
nd, nf = 4 * B, 8 * k.conv2_wino_filter_groups(B)
buf = torch.zeros(2 * (nd + nf), dtype=torch.int64, device="cuda")
eng.train(20)
torch.cuda.synchronize()
k.set_conv2_bwd_wino_prof(buf.data_ptr())
for rep in range(3):
    buf.zero_()
    eng.train(1)
    torch.cuda.synchronize()
    st = buf.view(-1, 2).cpu().numpy().astype(np.float64)
    t0 = st[:, 0].min()
    rel = (st - t0) / 100.0
    print(f"rep {rep}: launch span {rel[:, 1].max():.2f} us")
    for name, lo, hi in (("data", 0, nd), ("filter", nd, nd + nf)):
        r = rel[lo:hi]
        d = r[:, 1] - r[:, 0]
        print(f"  {name:7s} n={len(r):4d} start {r[:, 0].min():6.2f} med {np.median(r[:, 0]):6.2f} "
              f"max {r[:, 0].max():6.2f} | end med {np.median(r[:, 1]):6.2f} max {r[:, 1].max():6.2f}"
              f" | dur med {np.median(d):6.2f} min {d.min():6.2f} max {d.max():6.2f}", flush=True)
k.set_conv2_bwd_wino_prof(0)
