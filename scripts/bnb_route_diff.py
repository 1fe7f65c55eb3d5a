"""Debug lab: ResNet-18 bf16, one forward + backward per BatchNorm-backward
route (MTA_BNB_MODES, e.g. "0,1"), every parameter gradient's relative
difference to the first route, in model order.
    python scripts/bnb_route_diff.py [--hw 32] [--batch 32]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpi_tensorflow_amd import config as C
from mpi_tensorflow_amd.ops import functional as Fn
from mpi_tensorflow_amd.runtime.generic_engine import GenericEngine
from mpi_tensorflow_amd.utils.data import synthetic_rows

ap = argparse.ArgumentParser()
ap.add_argument("--hw", type=int, default=32)
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--modes", default="off,on,on-ignore")
a = ap.parse_args()
x, y = synthetic_rows("train", 0, 4 * a.batch, shape=(a.hw, a.hw, 3))
res = {}
for mode in a.modes.split(","):
    Fn.set_bn_bwd_epilogue(mode.startswith("on"))
    os.environ["MTA_BNB_IGNORE"] = "1" if mode.endswith("ignore") else "0"
    eng = GenericEngine(C.TrainConfig(model="resnet18", batch_size=a.batch, dtype="bf16",
                                      graph=False).validate(), x, y, torch.device("cuda:0"))
    eng.forward_backward_gpu()
    torch.cuda.synchronize()
    res[mode] = {k: v.clone() for k, v in eng.layout.views(eng.grads).items()}
modes = list(res)
base = res[modes[0]]
for k in base:
    errs = [((res[m][k] - base[k]).norm() / base[k].norm().clamp_min(1e-20)).item() for m in modes[1:]]
    print(f"{k:14s} " + " ".join(f"{m}={e:.2e}" for m, e in zip(modes[1:], errs)))
