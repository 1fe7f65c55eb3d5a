"""First-replay cost of a freshly captured MNIST training graph, with and
without hipGraphUpload after instantiation (the bench's driver window times
a graph whose first launch would otherwise happen inside the timing).
    python scripts/graph_first_launch.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpi_tensorflow_amd import config as C
from mpi_tensorflow_amd.ops import native, stream_handle
from mpi_tensorflow_amd.runtime.mnist_engine import NativeMnistEngine
from mpi_tensorflow_amd.utils.data import synthetic_rows


def run(upload: bool):
    x, y = synthetic_rows("train", 0, 4096)
    e = NativeMnistEngine(C.TrainConfig(graph_steps=10).validate(), x, y, torch.device("cuda"))
    e.train(5)
    torch.cuda.synchronize()
    g = e._graph(10)
    if upload:
        native().graph_upload(g.raw_cuda_graph_exec(), stream_handle())
    torch.cuda.synchronize()
    ts = []
    for _ in range(4):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        ts.append(round(a.elapsed_time(b) * 1000.0, 1))
    print(f"upload={upload}: replay us (10 steps each) {ts}", flush=True)


if __name__ == "__main__":
    run(False)
    run(True)
    run(False)
