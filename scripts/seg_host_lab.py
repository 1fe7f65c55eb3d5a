"""Host vs device time of the ResNet-18 bf16 multi-rank step replays (emulated
8-rank ring, no link cost): is the segmented capture host-bound?

    python scripts/seg_host_lab.py [--plan geo:8] [--graph-steps 10] [--reps 5]

Prints, per replay call of G steps: host seconds spent issuing it, and the
device time of all calls (events)."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mpi_tensorflow_amd import config as C  # noqa: E402
from mpi_tensorflow_amd.parallel.comm import EmulatedDeviceComm  # noqa: E402
from mpi_tensorflow_amd.runtime.generic_engine import GenericEngine  # noqa: E402
from mpi_tensorflow_amd.utils.data import synthetic_images_torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--plan", default="geo:8")
ap.add_argument("--graph-steps", type=int, default=10)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--n1", action="store_true", help="no sync at all (N = 1)")
ap.add_argument("--torch-events", action="store_true", help="default (system-fence) events")
ap.add_argument("--side-stream", action="store_true", help="replay on a non-default stream")
a = ap.parse_args()
if a.torch_events:
    import mpi_tensorflow_amd.parallel.overlap as OV

    OV.USE_DEV_EVENTS = False

dev = torch.device("cuda:0")
x, y = synthetic_images_torch(256, (224, 224, 3), seed=1)
cfg = C.TrainConfig(model="resnet18", dtype="bf16", batch_size=32, graph_steps=a.graph_steps,
                    bucket_plan=a.plan).validate()
comm = None if a.n1 else EmulatedDeviceComm(8, 0.0, 100000.0, 32)
eng = GenericEngine(cfg, x.numpy(), y.numpy(), dev, comm=comm, force_sync=not a.n1)
eng.capture(a.graph_steps)
eng.train(a.graph_steps)
torch.cuda.synchronize()
g = eng._graph(a.graph_steps)
side = torch.cuda.Stream()
if a.side_stream:
    side.wait_stream(torch.cuda.current_stream())
    torch.cuda.set_stream(side)
t0 = torch.cuda.Event(enable_timing=True)
t1 = torch.cuda.Event(enable_timing=True)
host = []
t0.record()
for _ in range(a.reps):
    h = time.perf_counter()
    g.replay()
    host.append(time.perf_counter() - h)
t1.record()
torch.cuda.synchronize()
dev_ms = t0.elapsed_time(t1) / (a.reps * a.graph_steps)
print(f"plan={a.plan if not a.n1 else 'n1'} torch_events={a.torch_events} "
      f"side_stream={a.side_stream} G={a.graph_steps} device {dev_ms * 1000:.1f} us/step; "
      f"host per replay call {[round(h * 1e3, 2) for h in host]} ms "
      f"({1e6 * sum(host) / (a.reps * a.graph_steps):.1f} us/step)")
