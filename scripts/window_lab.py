"""How the driver's short timed window relates to the steady state (lab):
MNIST fp32 as bench.py builds it, a prewarm of the given kind, 5 warm-up
steps, then 30 back-to-back 20-step windows, each bracketed by a device
synchronize and timed on the host clock as bench.py times its window.
    python scripts/window_lab.py [--prewarm eval|none|idle] [--ms 1000]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from mpi_tensorflow_amd import config as C  # noqa: E402
from mpi_tensorflow_amd.runtime.mnist_engine import make_engine  # noqa: E402
from mpi_tensorflow_amd.utils.data import load_mnist_shard  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--prewarm", default="eval", choices=("eval", "none", "idle"))
ap.add_argument("--ms", type=float, default=1000.0)
ap.add_argument("--windows", type=int, default=30)
ap.add_argument("--first", default="plain", choices=("plain", "upload", "replay"),
                help="before the warm-up: nothing, hipGraphUpload of the 20-step graph, or one "
                     "replay of it on snapshotted (restored) state")
a = ap.parse_args()
cfg = C.TrainConfig(batch_size=64).validate()
sh = load_mnist_shard(0, 1, synthetic=True, seed=cfg.seed)
dev = torch.device("cuda")
eng = make_engine(cfg, sh.train_x, sh.train_y, dev, 0, 1, None)
eng.capture(5)
eng.capture(20)
if a.prewarm == "eval":
    bench.prewarm(eng, sh.test_x, sh.test_y, a.ms)
elif a.prewarm == "idle":
    time.sleep(a.ms / 1000.0)
torch.cuda.synchronize()
g20 = eng._graph(20)
if a.first == "upload":
    from mpi_tensorflow_amd.ops import native, stream_handle
    native().graph_upload(g20.raw_cuda_graph_exec(), stream_handle())
elif a.first == "replay":
    snap = (eng.params.clone(), eng.mom.clone(), eng.step_dev.clone())
    g20.replay()
    eng.exe.join(__import__("mpi_tensorflow_amd.ops", fromlist=["stream_handle"]).stream_handle())
    eng.params.copy_(snap[0])
    eng.mom.copy_(snap[1])
    eng.step_dev.copy_(snap[2])
torch.cuda.synchronize()
eng.train(5)
torch.cuda.synchronize()
out = []
for w in range(a.windows):
    t0 = time.perf_counter()
    eng.train(20)
    torch.cuda.synchronize()
    out.append(1e6 * (time.perf_counter() - t0) / 20)
print(f"prewarm={a.prewarm} {a.ms:.0f} ms first={a.first}: us/step per 20-step window: "
      + " ".join(f"{v:.1f}" for v in out), flush=True)
