"""Per-role block timeline of the bf16 merged conv2 backward launch (lab):
eager training steps with per-block clock stamps (100 MHz), then for each
role the start / end spread relative to the launch's first block start.
    python scripts/c2b_stamps.py"""
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
cfg = C.TrainConfig(batch_size=B, dtype="bf16", graph=False).validate()
sh = load_mnist_shard(0, 1, synthetic=True, seed=cfg.seed)
eng = make_engine(cfg, sh.train_x, sh.train_y, torch.device("cuda"), 0, 1, None)
k = native().mnist
G = k.conv2_filter_groups_bf16(B)
nc2, nd = 25 * G, k.conv2_bwd_conv1_rows_bf16(B)
buf = torch.zeros(2 * 4096, dtype=torch.int64, device="cuda")
eng.train(20)
torch.cuda.synchronize()
k.set_conv2_bwd_prof_bf16(buf.data_ptr())
for rep in range(3):
    buf.zero_()
    eng.train(1)
    torch.cuda.synchronize()
    allv = buf.cpu().numpy()
    st = allv.reshape(-1, 2)
    nb = int((st[:, 1] > 0).sum())
    st = st[:nb]
    ph = allv[2 * nb:2 * nb + 8 * nd].reshape(nd, 8)[:, :5]
    t0 = st[:, 0].min()
    rel = (st - t0) / 100.0  # us
    print(f"rep {rep}: {nb} blocks, launch span {rel[:, 1].max():.2f} us")
    d0, f0 = 0, nd  # role order: data, filter, FC SGD
    for name, lo, hi in (("filter", f0, f0 + nc2), ("data+conv1", d0, d0 + nd),
                         ("fc-sgd", nc2 + nd, nb)):
        r = rel[lo:hi]
        if len(r) == 0:
            continue
        d = r[:, 1] - r[:, 0]
        if name.startswith("data"):
            seg = (ph - st[lo:hi, :1]) / 100.0  # phase ends relative to the block start
            seg = np.where(ph > 0, seg, np.nan)
            med = np.nanmedian(seg, axis=0)
            print("    data phase ends (median us from block start): staged %.2f  K loop %.2f  "
                  "dA1 %.2f  conv1 staged %.2f  conv1 GEMM %.2f" % tuple(med))
        print(f"  {name:11s} n={len(r):4d} start {r[:, 0].min():6.2f}..{r[:, 0].max():6.2f}  "
              f"end {np.percentile(r[:, 1], 50):6.2f}/{r[:, 1].max():6.2f}  dur med {np.median(d):6.2f} "
              f"max {d.max():6.2f}", flush=True)
k.set_conv2_bwd_prof_bf16(0)
