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

import numpy as np
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


_M64 = (1 << 64) - 1


def _splitmix64_np(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


def replica_hash(t: torch.Tensor) -> int:
    """Bitwise replica fingerprint of a 32-bit tensor: sum over i (mod 2^64)
    of splitmix64((i << 32) | raw_word_i).  Sensitive to every bit, to sign
    flips and to permutations (position-keyed), exact (integer arithmetic).
    GPU tensors hash on the device (csrc/kernels/sgd.hip hash_words_kernel,
    one 8-byte read back); CPU tensors hash here with the same function."""
    x = t.detach().contiguous().view(-1)
    if x.element_size() != 4:
        raise ValueError("replica_hash hashes 32-bit words")
    if x.is_cuda:
        from ..ops import native, ptr, stream_handle

        out = torch.empty(1, dtype=torch.int64, device=x.device)
        native().optim.hash_words(ptr(x), x.numel(), ptr(out), stream_handle())
        return int(out.item()) & _M64
    w = x.view(torch.int32).numpy().view(np.uint32).astype(np.uint64)
    i = np.arange(w.size, dtype=np.uint64)
    h = _splitmix64_np((i << np.uint64(32)) | w)
    with np.errstate(over="ignore"):
        return int(np.sum(h, dtype=np.uint64)) & _M64


def replicas_identical(t: torch.Tensor) -> bool:
    """True iff every rank's tensor hashes identically (gloo host group)."""
    import torch.distributed as dist

    h = replica_hash(t)
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() <= 1:
        return True
    v = torch.tensor([h - (1 << 64) if h >= (1 << 63) else h], dtype=torch.int64)
    lo, hi = v.clone(), v.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    return bool(lo.item() == hi.item())
