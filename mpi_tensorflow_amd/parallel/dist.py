"""Process-group bootstrap: rank discovery, device binding, gloo/RCCL init.

The reference takes `MPI.COMM_WORLD`, `Get_rank()`, `Get_size()`
(`/root/reference/mpipy.py:208-210`) and never binds a GPU, so every rank
lands on `/GPU:0` (quirk Q13).  Here:

* rank / world / local rank come from torchrun (`RANK`, `WORLD_SIZE`,
  `LOCAL_RANK`), Open MPI (`OMPI_COMM_WORLD_*`), MPICH/Hydra PMI
  (`PMI_RANK`, `PMI_SIZE`, `MPI_LOCALRANKID`) or Slurm (`SLURM_PROCID`, ...),
  so both `torchrun` and `mpirun` launches work;
* each rank binds GPU `local_rank` (one process per GPU);
* `torch.distributed` is initialised with a CPU gloo group (bootstrap,
  barriers, timing max-reduce, CPU training) and, on GPU, the device
  collectives go through the native RCCL communicator in `parallel/comm.py`
  (bootstrapped over the same TCPStore) with torch's `nccl` (= RCCL)
  backend as the fallback.
"""

from __future__ import annotations

import dataclasses
import datetime
import os
from typing import Optional

import torch
import torch.distributed as dist


@dataclasses.dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    local_world: int = 1
    launcher: str = "none"

    @property
    def is_root(self) -> bool:
        return self.rank == 0


def _env_int(*names: str) -> Optional[int]:
    for n in names:
        v = os.environ.get(n)
        if v not in (None, ""):
            try:
                return int(v)
            except ValueError:
                pass
    return None


def discover() -> DistInfo:
    """Rank layout from the launcher's environment (torchrun > MPI > Slurm)."""
    if _env_int("RANK") is not None and _env_int("WORLD_SIZE") is not None:
        r, w = _env_int("RANK"), _env_int("WORLD_SIZE")
        lr = _env_int("LOCAL_RANK")
        lw = _env_int("LOCAL_WORLD_SIZE")
        return DistInfo(r, w, lr if lr is not None else r, lw if lw is not None else w, "torchrun")
    if _env_int("OMPI_COMM_WORLD_RANK") is not None:
        r = _env_int("OMPI_COMM_WORLD_RANK")
        w = _env_int("OMPI_COMM_WORLD_SIZE") or 1
        lr = _env_int("OMPI_COMM_WORLD_LOCAL_RANK")
        lw = _env_int("OMPI_COMM_WORLD_LOCAL_SIZE")
        return DistInfo(r, w, lr if lr is not None else r, lw if lw is not None else w, "openmpi")
    if _env_int("PMI_RANK") is not None:
        r = _env_int("PMI_RANK")
        w = _env_int("PMI_SIZE") or 1
        lr = _env_int("MPI_LOCALRANKID", "PMI_LOCAL_RANK")
        lw = _env_int("MPI_LOCALNRANKS", "PMI_LOCAL_SIZE")
        return DistInfo(r, w, lr if lr is not None else r, lw if lw is not None else w, "pmi")
    if _env_int("SLURM_PROCID") is not None and _env_int("SLURM_NTASKS") is not None:
        r, w = _env_int("SLURM_PROCID"), _env_int("SLURM_NTASKS")
        lr = _env_int("SLURM_LOCALID")
        lw = _env_int("SLURM_NTASKS_PER_NODE")
        return DistInfo(r, w, lr if lr is not None else r, lw if lw is not None else w, "slurm")
    return DistInfo()


_INFO: Optional[DistInfo] = None


def info() -> DistInfo:
    return _INFO if _INFO is not None else discover()


def init(device: str = "auto", timeout_s: float = 600.0) -> DistInfo:
    """Initialises the process group (idempotent).  Returns the DistInfo.

    A gloo group is always created when world > 1: it carries the RCCL
    unique-id exchange, barriers and host-side reductions.  Device binding:
    `torch.cuda.set_device(local_rank)` when running on GPU.
    """
    global _INFO
    di = discover()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    # dmabuf-only IPC on this driver stack (see environment notes)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    on_gpu = resolve_device(device).type == "cuda"
    if on_gpu:
        ndev = torch.cuda.device_count()
        if ndev == 0:
            raise RuntimeError("GPU requested but no device is visible")
        torch.cuda.set_device(di.local_rank % ndev)
    if di.world > 1 and not dist.is_initialized():
        dist.init_process_group(
            backend="gloo",
            init_method=f"tcp://{os.environ['MASTER_ADDR']}:{os.environ['MASTER_PORT']}",
            rank=di.rank,
            world_size=di.world,
            timeout=datetime.timedelta(seconds=timeout_s),
        )
    _INFO = di
    return di


def resolve_device(device: str = "auto") -> torch.device:
    if device in (None, "auto"):
        return torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")
    return torch.device(device)


def barrier() -> None:
    if dist.is_available() and dist.is_initialized():
        dist.barrier()


def allreduce_max_host(x: float) -> float:
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        t = torch.tensor([float(x)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())
    return float(x)


def allreduce_sum_host(x: float) -> float:
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        t = torch.tensor([float(x)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return float(t.item())
    return float(x)


def shutdown() -> None:
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
