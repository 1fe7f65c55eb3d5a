"""Calibrates the ResNet-18 synthetic task (utils/data.py synthetic_images_torch):
trains fp32 and bf16 on the GPU and prints the loss curve and the held-out
accuracy.  python scripts/resnet_task_cal.py [--steps 300] [--noise 0.35]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpi_tensorflow_amd import config as C
from mpi_tensorflow_amd.runtime.generic_engine import GenericEngine
from mpi_tensorflow_amd.utils.data import synthetic_images_torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--rows", type=int, default=2048)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--noise", type=float, nargs="+", default=[0.35])
    ap.add_argument("--dtypes", nargs="+", default=["fp32", "bf16"])
    a = ap.parse_args()
    dev = torch.device("cuda")
    for nz in a.noise:
        t0 = time.time()
        tx, ty = synthetic_images_torch(a.rows, (224, 224, 3), device=dev, noise=nz)
        ex, ey = synthetic_images_torch(512, (224, 224, 3), device=dev, split="test", noise=nz)
        tx, ty, ex, ey = tx.cpu().numpy(), ty.numpy(), ex.cpu().numpy(), ey.numpy()
        print(f"noise {nz}: data {time.time() - t0:.1f}s", flush=True)
        for dt in a.dtypes:
            cfg = C.TrainConfig(model="resnet18", batch_size=a.batch, dtype=dt, graph_steps=25).validate()
            e = GenericEngine(cfg, tx, ty, dev)
            curve = []
            t0 = time.time()
            for k in range(a.steps // 25):
                e.train(25)
                curve.append(round(e.loss_value(), 3))
            torch.cuda.synchronize()
            err = e.evaluate(ex, ey)
            print(f"  {dt}: acc {100 - err:.2f}% after {e.step} steps ({time.time() - t0:.1f}s) "
                  f"loss curve {curve}", flush=True)


if __name__ == "__main__":
    main()
