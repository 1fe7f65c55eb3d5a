"""First-replay cost of a captured MNIST training graph (1 GPU).

The driver times `bench.py --steps 20 --warmup 5`: the 20-step graph is
captured outside the timing but REPLAYED for the first time inside it.  This
script times consecutive replays of the same graph (wall clock, bracketed by
device synchronizes like bench.py) and the host time of each replay() call.
    python scripts/replay_lab.py [--steps 20] [--dtype fp32]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mpi_tensorflow_amd import config as C  # noqa: E402
from mpi_tensorflow_amd.runtime.mnist_engine import make_engine  # noqa: E402
from mpi_tensorflow_amd.utils.data import load_mnist_shard  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--dtype", default="fp32")
ap.add_argument("--reps", type=int, default=6)
a = ap.parse_args()
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
cfg = C.TrainConfig(dtype=a.dtype).validate()
shard = load_mnist_shard(0, 1, synthetic=True, seed=cfg.seed)
eng = make_engine(cfg, shard.train_x, shard.train_y, dev, 0, 1, None)
eng.capture(5)
eng.capture(a.steps)
eng.train(5)
torch.cuda.synchronize()
for rep in range(a.reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.train(a.steps)
    th = time.perf_counter()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    print(f"replay {rep}: {1e6 * (t1 - t0) / a.steps:8.2f} us/step  "
          f"host {1e6 * (th - t0):8.1f} us  total {1e6 * (t1 - t0):8.1f} us", flush=True)
# long run for the steady state
torch.cuda.synchronize()
t0 = time.perf_counter()
eng.train(1000)
torch.cuda.synchronize()
print(f"1000 steps: {1e3 * (time.perf_counter() - t0):8.2f} us/step")
