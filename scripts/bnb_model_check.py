"""Debug lab: one ResNet-18 bf16 forward + backward with MTA_BNB_CHECK=1 - every
BatchNorm backward that takes the dgrad-epilogue sums also runs its own
statistics pass and prints both sums' relative difference.
    MTA_BNB_CHECK=1 python scripts/bnb_model_check.py [--hw 32] [--batch 32]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpi_tensorflow_amd import config as C
from mpi_tensorflow_amd.runtime.generic_engine import GenericEngine
from mpi_tensorflow_amd.utils.data import synthetic_rows

ap = argparse.ArgumentParser()
ap.add_argument("--hw", type=int, default=32)
ap.add_argument("--batch", type=int, default=32)
a = ap.parse_args()
x, y = synthetic_rows("train", 0, 4 * a.batch, shape=(a.hw, a.hw, 3))
eng = GenericEngine(C.TrainConfig(model="resnet18", batch_size=a.batch, dtype="bf16",
                                  graph=False).validate(), x, y, torch.device("cuda:0"))
eng.forward_backward_gpu()
torch.cuda.synchronize()
