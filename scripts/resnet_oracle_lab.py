"""ResNet-18 held-out accuracy of the native engines vs the PyTorch-op oracle
at several run lengths, with the oracle's MIOpen algorithms deterministic or
not: how far the oracle itself moves with summation order
(tests/test_accuracy_gpu.py pins native vs oracle).

  python scripts/resnet_oracle_lab.py --steps 600,1200
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mpi_tensorflow_amd import config as C  # noqa: E402
from mpi_tensorflow_amd.runtime.generic_engine import GenericEngine  # noqa: E402
from mpi_tensorflow_amd.utils.data import synthetic_images_torch  # noqa: E402


def run(dev, task, dtype, steps, oracle, det):
    tx, ty, ex, ey = task
    cfg = C.TrainConfig(model="resnet18", batch_size=32, dtype=dtype, graph=not oracle,
                        graph_steps=25).validate()
    with torch.backends.cudnn.flags(enabled=True, benchmark=False, deterministic=det):
        e = GenericEngine(cfg, tx, ty, dev, oracle=oracle)
        accs = {}
        done = 0
        for s in steps:
            while done < s:  # progress lines (a silent GPU run reads as hung)
                k = min(100, s - done)
                e.train(k)
                done += k
                torch.cuda.synchronize()
                print(f"  {dtype} oracle={oracle} det={det}: {done} steps", flush=True)
            accs[s] = 100.0 - e.evaluate(ex, ey)
    del e
    torch.cuda.empty_cache()
    return accs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", default="600,1200")
    ap.add_argument("--rows", type=int, default=4096)
    a = ap.parse_args()
    steps = [int(s) for s in a.steps.split(",")]
    dev = torch.device("cuda:0")
    tx, ty = synthetic_images_torch(a.rows, (224, 224, 3), device=dev)
    ex, ey = synthetic_images_torch(1024, (224, 224, 3), device=dev, split="test")
    task = (tx.cpu().numpy(), ty.numpy(), ex.cpu().numpy(), ey.numpy())
    for name, dtype, oracle, det in (("oracle", "fp32", True, False),
                                     ("oracle", "fp32", True, False),
                                     ("native", "fp32", False, False),
                                     ("native", "bf16", False, False),
                                     ("oracle det", "fp32", True, True)):
        accs = run(dev, task, dtype, steps, oracle, det)
        print(f"{name:14s} {dtype}: " + "  ".join(f"{s}: {v:.2f}%" for s, v in accs.items()),
              flush=True)


if __name__ == "__main__":
    main()
