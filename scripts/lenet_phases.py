"""Per-phase time of the fused LeNet-5 image kernel (profiling aid): times
the kernel stopped after each phase, in a 50-launch hipGraph."""
import sys

import torch

sys.path.insert(0, ".")
from mpi_tensorflow_amd import config as C  # noqa: E402
from mpi_tensorflow_amd.ops import native, stream_handle  # noqa: E402
from mpi_tensorflow_amd.runtime.lenet_engine import NativeLenetEngine  # noqa: E402
from mpi_tensorflow_amd.utils.data import synthetic_rows  # noqa: E402

x, y = synthetic_rows("train", 0, 2048, shape=(32, 32, 3))
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
e = NativeLenetEngine(C.TrainConfig(model="lenet5", batch_size=B).validate(), x, y,
                      torch.device("cuda"))
e.train(5)
Cn = native()
prev = 0.0
for stop in (0, 1, 2, 10, 11, 12, 3, 4, 5, 6, 99):  # 10-12: D / E / F inside 3
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(50):
            Cn.lenet_image_phase(e.ptrs, stop, stream_handle())
    g.replay()
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(4):
        g.replay()
    t1.record()
    t1.synchronize()
    us = t0.elapsed_time(t1) * 1000 / 200
    print(f"stop after phase {stop:2d}: {us:7.2f} us  (+{us - prev:6.2f})", flush=True)
    prev = us
