"""Debug: captured-graph LeNet vs eager twin under different call patterns."""
import sys
sys.path.insert(0, "/root/repo")
import torch
from mpi_tensorflow_amd import config as C
from mpi_tensorflow_amd.runtime.generic_engine import GenericEngine
from mpi_tensorflow_amd.utils.data import synthetic_image_shard

dev = torch.device("cuda:0")
sh = synthetic_image_shard(0, 1, 8192, 2048, (32, 32, 3), seed=1)
mk = lambda g: GenericEngine(C.TrainConfig(model="lenet5", graph=g, graph_steps=10).validate(),
                             sh.train_x, sh.train_y, dev)


def run(name, pattern):
    a, b = mk(False), mk(True)
    bad = None
    for i, k in enumerate(pattern):
        a.train(k)
        b.train(k)
        torch.cuda.synchronize()
        va, vb = a.layout.views(a.params.detach()), b.layout.views(b.params.detach())
        worst = max(((va[n] - vb[n]).abs().max().item(), n) for n in va)
        if worst[0] > 1e-3 and bad is None:
            bad = (i, b.step, worst)
    print(f"{name}: first divergence {bad}", flush=True)


run("30s", [30] * 6)
run("23 then 20s (warm-up + 2 replays, then pure replays)", [23] + [20] * 8)
run("replays with eager remainders", [25] * 8)
