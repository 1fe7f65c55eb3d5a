"""Data-parallel synchronisation strategies.

Reference (`Cnn.bcast_parameters`, `/root/reference/mpipy.py:95-153`, called
every 50 steps at `:87-91`): each rank `eval()`s its four weight tensors to
host numpy, `comm.Gather`s them to rank 0, rank 0 takes `np.mean` and
assigns it through NEW graph ops each call.  Biases and momentum are never
averaged and non-root ranks never receive the mean (quirk Q11); the graph
grows by ~6.65 MB of constants per call (Q12).

Strategies here (all operate in place on the flat device buffers):

* `grad`      - per-step gradient all-reduce inside the training step (the
                default; done by the engines, see runtime/mnist_engine.py).
* `param_avg` - every `sync_every` steps: ONE all-reduce of the whole flat
                parameter buffer, divided by world size, on ALL ranks.
* root-only   - `--reference-quirks`: reduce of the four weight tensors to
                rank 0 only, rank 0 keeps the mean, others are untouched
                (faithful to Q11).
"""

from __future__ import annotations

from typing import Iterable

import torch

from .comm import DeviceComm
from .flat import FlatLayout

REFERENCE_AVERAGED = ("conv1_weight", "conv2_weight", "fc1_weight", "fc2_weight")  # mpipy.py:121-127


@torch.no_grad()
def average_params(comm: DeviceComm, params: torch.Tensor) -> None:
    # `params` may be an autograd leaf (generic engine): work on its storage
    p = params.detach()
    comm.all_reduce_(p)
    p.mul_(1.0 / comm.size)


@torch.no_grad()
def average_params_root_only(comm: DeviceComm, layout: FlatLayout, params: torch.Tensor,
                             names: Iterable[str] = REFERENCE_AVERAGED) -> None:
    views = layout.views(params.detach())
    for n in names:
        v = views[n]
        buf = v.detach().clone().contiguous().view(-1)  # reduce may scratch non-root buffers
        comm.reduce_(buf, root=0)
        if comm.rank == 0:
            v.copy_(buf.view(v.shape) / comm.size)


def replica_checksum(params: torch.Tensor) -> float:
    """Cheap cross-replica consistency probe (sum of |w| in float64)."""
    return float(params.detach().double().abs().sum().item())
