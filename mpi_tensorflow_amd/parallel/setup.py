"""One communicator set-up for every entry point (`bench.py` and the
`mpipy.py` Trainer), so the one-script API trains with the same sync the
benchmark measured.

The reference has exactly one communicator, `MPI.COMM_WORLD`
(/root/reference/mpipy.py:208-210), used for the Scatter of the shards and the
Gather-to-root weight averaging (`:121-137`).  Here a run gets:

* `comm`  - the device communicator of parallel/comm.py `make_comm` (RCCL over
  xGMI, the shared-memory one when ranks share GPUs, gloo on the CPU), for
  world > 1 whenever the ranks sync at all;
* `xcomm` - on one node with one GPU per rank, for the MNIST CNN and LeNet-5
  with `--comm auto`: the xGMI peer-to-peer communicator as an extra sync
  candidate - only after it passed the exactness check
  (`comm.xgmi_exactness_check`: integer data, bitwise equal to the exact sum
  and to `comm`'s sum).  The engine's auto-tune then also compares one trial
  step of each xGMI schedule with a step synced over `comm`
  (runtime/mnist_engine.py `_xgmi_step_matches`, runtime/lenet_engine.py
  `tune_schedule`).

`health_vote` is the run-time half: the xGMI kernels never hang (a missing
peer sets a sticky error bit and the later barriers stop waiting), so every
entry point votes on that bit at its synchronisation points and stops on
every rank when any rank saw it.
"""

from __future__ import annotations

import dataclasses
from typing import Optional

import torch

from .. import config as C
from . import comm as CM
from . import dist as D


def comm_capacity_bytes(cfg: C.TrainConfig) -> int:
    """Largest per-rank contribution of one collective of this model's step,
    rounded up to 1 MiB: the capacity a shared-memory communicator needs.
    That is the whole flat fp32 gradient / parameter buffer, or for the MNIST
    factor schedule (csrc/mnist_executor.cpp train_step_factors) one rank's
    FC-factor slice a2 / dh / hd / dlog, B x (3136 + 2 x 512 + 10) floats,
    when that is larger (B > ~400)."""
    if cfg.model == "mnist_cnn":
        from ..models import mnist_cnn as M

        total = M.layout().total
        total = max(total, cfg.batch_size * (M.FC1_IN + 2 * M.FC1_OUT + 10))
    else:
        from ..models.generic import make_model

        total = make_model(cfg.model).layout.total
    return ((4 * total + (1 << 20) - 1) >> 20) << 20


def wants_comm(cfg: C.TrainConfig, world: int) -> bool:
    """A device communicator exists when ranks exchange anything: per-step
    gradient sync or the reference's periodic parameter averaging."""
    return world > 1 and cfg.sync in ("grad", "param_avg")


def wants_xgmi_candidate(cfg: C.TrainConfig, comm_kind: str, no_xgmi: bool = False) -> bool:
    """The xGMI peer-to-peer syncs are tuned next to RCCL's for the MNIST CNN
    and LeNet-5 (the fused executors) when the user left the communicator to
    `auto`, RCCL is what auto chose (one GPU per rank; ranks sharing GPUs use
    the host shared-memory path) and the ranks sync gradients every step.
    Pure: both entry points decide with it (tests/test_comm_setup_cpu.py)."""
    return (cfg.comm == "auto" and not no_xgmi and cfg.model in ("mnist_cnn", "lenet5")
            and cfg.sync == "grad" and comm_kind == "rccl-native")


@dataclasses.dataclass
class CommSet:
    comm: Optional[CM.DeviceComm] = None
    xcomm: Optional[CM.XgmiDeviceComm] = None
    xgmi_status: str = "n/a"  # passed / dropped: <why> / not set up: <why> / n/a

    def report(self) -> dict:
        return {"comm": getattr(self.comm, "kind", "none"),
                "xgmi_comm": getattr(self.xcomm, "kind", None),
                "xgmi_gate": self.xgmi_status}


def setup_comms(di: D.DistInfo, device: torch.device, cfg: C.TrainConfig,
                no_xgmi: bool = False, xgmi_timeout_s: float = 20.0) -> CommSet:
    """Collective over the ranks (every rank takes the same branches)."""
    out = CommSet()
    if not wants_comm(cfg, di.world):
        return out
    out.comm = CM.make_comm(di, device, cfg.comm, shm_capacity=comm_capacity_bytes(cfg),
                            timeout_s=cfg.collective_timeout_s)
    if isinstance(out.comm, CM.XgmiDeviceComm):  # --comm xgmi: gated inside make_comm
        out.xgmi_status = out.comm.gate
    elif (device.type == "cuda"
          and wants_xgmi_candidate(cfg, getattr(out.comm, "kind", ""), no_xgmi)):
        out.xcomm = CM.make_xgmi_comm(di, device, min(xgmi_timeout_s, cfg.collective_timeout_s),
                                      ref=out.comm)
        out.xgmi_status = CM.last_xgmi_status
    return out


def xgmi_comms(*objs):
    """The xGMI communicators among `objs` (communicators or engines)."""
    seen = []
    for o in objs:
        for c in (o, getattr(o, "comm", None), getattr(o, "xcomm", None)):
            if isinstance(c, CM.XgmiDeviceComm) and not any(c is s for s in seen):
                seen.append(c)
    return seen


def health_vote(*objs) -> int:
    """Collective: the largest sticky xGMI error word over the ranks and the
    xGMI communicators among `objs` (0 = healthy; syncs the device).  Every
    rank gets the same value, so every rank stops together."""
    bad = 0
    for c in xgmi_comms(*objs):
        bad = max(bad, c.error())
    return int(D.allreduce_max_host(float(bad)))


def check_health(where: str, *objs) -> None:
    """Raises on every rank when any rank's xGMI barrier timed out: the later
    barriers of that communicator no longer wait, so training on would read
    peers' buffers unsynchronized."""
    bad = health_vote(*objs)
    if bad:
        raise RuntimeError(f"xGMI communicator failed ({where}): a peer barrier timed out "
                           f"(error word {bad}); its collectives are no longer synchronised")
