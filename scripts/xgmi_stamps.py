"""Per-phase block timeline of the MNIST xGMI step launch (xgmi_step_kernel,
lab) on one GPU as an emulated N-rank communicator:
    python scripts/xgmi_stamps.py [--emulate 0,0,8] [--sched xgmi-step]
Stamps (100 MHz): 0 start, 1 before barrier 0 (FC: epoch taken; conv: slab
sums written), 2 after barrier 0, 3 before barrier 1 (FC: segment summed +
SGD; conv: rank sums + SGD + Winograd), 4 after barrier 1, 5 end (FC: gather
done)."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpi_tensorflow_amd import config as C  # noqa: E402
from mpi_tensorflow_amd.ops import native  # noqa: E402
from mpi_tensorflow_amd.parallel.comm import XgmiDeviceComm  # noqa: E402
from mpi_tensorflow_amd.runtime.mnist_engine import make_engine  # noqa: E402
from mpi_tensorflow_amd.utils.data import load_mnist_shard  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--emulate", default="0,0,8")
ap.add_argument("--sched", default="xgmi-step")
a = ap.parse_args()
f = [float(v) for v in a.emulate.split(",")]
B = 64
cfg = C.TrainConfig(batch_size=B, graph=False, sync_schedule=a.sched).validate()
sh = load_mnist_shard(0, 1, synthetic=True, seed=cfg.seed)
xe = XgmiDeviceComm.emulated(int(f[2]), f[0], f[1])
eng = make_engine(cfg, sh.train_x, sh.train_y, torch.device("cuda"), 0, 1, xe, force_sync=True)
k = native().mnist
buf = torch.zeros(6 * 4096, dtype=torch.int64, device="cuda")
eng.train(20)
torch.cuda.synchronize()
k.set_xgmi_step_prof(buf.data_ptr())
for rep in range(3):
    buf.zero_()
    eng.train(1)
    torch.cuda.synchronize()
    raw = buf.view(-1, 6).cpu().numpy()
    used = raw[:, 5] > 0
    raw = raw[used]
    fc = (raw[:, 0] >> 60) == 1
    st = (raw & ((1 << 56) - 1)).astype(np.float64)
    t0 = st[:, 0].min()
    rel = (st - t0) / 100.0
    print(f"rep {rep}: {len(st)} blocks, launch span {rel[:, 5].max():.2f} us")
    for name, m in (("FC", fc), ("conv", ~fc)):
        r = rel[m]
        if len(r) == 0:
            continue
        med = np.median(r, axis=0)
        mx = r.max(axis=0)
        print(f"  {name:4s} n={len(r):4d} median stamps " + " ".join(f"{v:6.2f}" for v in med) +
              "   max " + " ".join(f"{v:6.2f}" for v in mx), flush=True)
k.set_xgmi_step_prof(0)
