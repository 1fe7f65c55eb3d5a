"""Native LeNet-5 engine (BASELINE config 4) on the fused kernels of
`csrc/kernels/lenet.hip` through the C++ `LenetExecutor`.

Same state and step contract as the other engines (flat fp32 param / grad /
momentum buffers in the parallel/flat.py layout, device step counter,
reference LR schedule + momentum SGD of /root/reference/mpipy.py:59-66,
batch offset (step * B) % (N - B) of :80, per-step gradient all-reduce for
DP), but a training step is two kernel launches (one workgroup per image for
the whole forward + backward, then the batch-level weight gradients + SGD)
instead of the ~37 of the generic op-by-op path, and G steps are captured
into one hipGraph.  The numerics oracle is the generic engine's CPU path
(models/generic.py LeNet5 on plain PyTorch ops).
"""

from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch

from .. import config as C
from ..models.generic import make_model
from ..ops import native, ptr, stream_handle
from ..parallel.comm import DeviceComm, XgmiDeviceComm
from ..utils.devcache import DeviceArrayCache
from ..utils.schedule import learning_rate

# the executor's xGMI sync modes (csrc/lenet_executor.h XGMI_*)
XGMI_MODES = C.XGMI_MODES
XGMI_MODE_IDS = {m: i for i, m in enumerate(XGMI_MODES)}

_OFFSETS = (("c1w", "c1_w"), ("c1b", "c1_b"), ("c2w", "c2_w"), ("c2b", "c2_b"), ("f1w", "f1_w"),
            ("f1b", "f1_b"), ("f2w", "f2_w"), ("f2b", "f2_b"), ("f3w", "f3_w"), ("f3b", "f3_b"))


class NativeLenetEngine:
    kind = "native-lenet5"

    def __init__(self, cfg: C.TrainConfig, train_x: np.ndarray, train_y: np.ndarray,
                 device: torch.device, rank: int = 0, world: int = 1,
                 comm: Optional[DeviceComm] = None, force_sync: bool = False,
                 xcomm: Optional[XgmiDeviceComm] = None):
        """xcomm: an exactness-gated xGMI communicator (parallel/setup.py) next
        to an RCCL `comm`: tune_schedule() times both syncs and keeps the
        faster (the xGMI one only after one trial step matched RCCL's)."""
        if device.type != "cuda":
            raise RuntimeError("NativeLenetEngine needs a GPU")
        if cfg.model != "lenet5":
            raise ValueError("NativeLenetEngine trains lenet5 only")
        if cfg.dtype != "fp32":
            raise NotImplementedError("the fused LeNet-5 kernels are fp32 (VALU convs over 3 / 6 "
                                      "channels); use the generic engine for bf16")
        self.cfg, self.device, self.rank, self.world, self.comm = cfg, device, rank, world, comm
        self.model = make_model("lenet5")
        self.layout = self.model.layout
        self.B = cfg.batch_size
        self.n_local = int(train_x.shape[0])
        if self.n_local <= self.B:
            raise ValueError("local shard must exceed the batch")
        if tuple(train_x.shape[1:]) != (32, 32, 3):
            raise ValueError(f"LeNet-5 input must be 32x32x3 NHWC, got {train_x.shape[1:]}")
        host = torch.zeros(self.layout.total)
        self.model.init_params(host, cfg.seed)
        dev = device
        self.params = host.to(dev)
        self.grads = torch.zeros(self.layout.total, device=dev)
        self.mom = torch.zeros(self.layout.total, device=dev)
        self.bn: Dict = {}
        self._eval_x = DeviceArrayCache()
        self.train_x = torch.from_numpy(np.ascontiguousarray(train_x, np.float32)).to(dev)
        self.train_y = torch.from_numpy(np.asarray(train_y).astype(np.int32)).to(dev)
        self.step = 0
        self.step_dev = torch.zeros(1, dtype=torch.int64, device=dev)
        self.lr_dev = torch.zeros(1, device=dev)
        self.correct_dev = torch.zeros(1, dtype=torch.int32, device=dev)
        self.grad_sync = cfg.sync == "grad" and world > 1 and comm is not None
        if force_sync and comm is not None:
            self.grad_sync = True
        C_ = native()
        self._C = C_
        na, nd, nc = C_.lenet_buffer_floats(self.B)
        self.acts = torch.zeros(na, device=dev)
        self.deltas = torch.zeros(nd, device=dev)
        self.convp = torch.zeros(nc, device=dev)
        self.loss_rows = torch.zeros(self.B, device=dev)
        p = C_.LenetPtrs()
        p.train_x, p.train_y = ptr(self.train_x), ptr(self.train_y)
        p.n_local, p.batch = self.n_local, self.B
        p.params, p.grads, p.mom = ptr(self.params), ptr(self.grads), ptr(self.mom)
        p.total = self.layout.total
        off = C_.LenetOffsets()
        for attr, name in _OFFSETS:
            setattr(off, attr, self.layout.offsets[name])
        p.off = off
        p.step, p.lr, p.correct = ptr(self.step_dev), ptr(self.lr_dev), ptr(self.correct_dev)
        p.acts, p.deltas, p.convp = ptr(self.acts), ptr(self.deltas), ptr(self.convp)
        p.loss_rows = ptr(self.loss_rows)
        p.base_lr, p.lr_decay, p.momentum = cfg.base_lr, cfg.lr_decay, cfg.momentum
        self.gb16 = None  # bf16 gradient wire staging (--grad-comm-dtype bf16)
        if cfg.grad_comm_dtype == "bf16" and self.grad_sync:
            if self.layout.total % 4:
                raise RuntimeError("bf16 gradient wire needs a flat buffer of 4k floats")
            self.gb16 = torch.zeros(self.layout.total, dtype=torch.bfloat16, device=dev)
            p.grad_bf16, p.gb16 = 1, ptr(self.gb16)
        self._native_comm = None
        self.xcomm = None
        self._sync = None  # the communicator the step syncs over (native handle)
        if self.grad_sync:
            self._native_comm = comm.native_handle
            if self._native_comm is None:
                raise RuntimeError("GPU grad sync needs the native RCCL communicator")
            if getattr(comm, "kind", "") == "host-staged":  # test comm: eager only
                comm.bases = [self.grads] + ([self.gb16] if self.gb16 is not None else [])
            self.xcomm = comm if isinstance(comm, XgmiDeviceComm) else xcomm
            if self.xcomm is not None:  # xGMI peer to peer: peers read the grads and
                # params, and (to make it whole) the sharded momentum
                if self.gb16 is not None:
                    raise ValueError("the xGMI communicator reduces fp32 grads only")
                self.xcomm.register(self.grads, self.params, self.mom)
                # receive slots [2 parities][N ranks][total] of the push sync
                # fused into the update launch (lenet.h PushArgs, replicated
                # momentum); the two-phase launch is the other xGMI form
                self.xrecv = torch.zeros(2 * self.xcomm.size * self.layout.total, device=dev)
                self.xcomm.register(self.xrecv)
                p.xrecv = ptr(self.xrecv)
                # the one-shot (pull) sync: double-buffered gradient slots
                # [2][total] read by every peer, and its completion counter
                self.xgrads2 = torch.zeros(2 * self.layout.total, device=dev)
                self.xcomm.register(self.xgrads2)
                self.xdone = torch.zeros(16, dtype=torch.int32, device=dev)
                p.xgrads2, p.xdone = ptr(self.xgrads2), ptr(self.xdone)
            self._sync = self._native_comm
            # connection setup of the collective, outside any capture (the
            # executor copies the pointer struct: made after xrecv is set)
            self.ptrs = p
            self.exe = C_.LenetExecutor(p)
            if self.xcomm is not None:
                self.exe.set_xgmi_mode(XGMI_MODE_IDS[cfg.xgmi_mode])
            self._native_comm.all_reduce(ptr(self.grads), ptr(self.grads), self.layout.total, 7, 0,
                                         stream_handle())
            torch.cuda.synchronize(dev)
        if not self.grad_sync:
            self.ptrs = p
            self.exe = C_.LenetExecutor(p)
        self.tune_log: Dict[str, Optional[float]] = {}
        self.tune_reject: Dict[str, str] = {}
        self.xgmi_step_check: Dict[str, float] = {}
        self._tuned = not (self.grad_sync and xcomm is not None and self.xcomm is xcomm
                           and cfg.graph and cfg.sync_schedule == "auto")
        self.use_graph = cfg.graph and getattr(comm, "kind", "") != "host-staged"
        self.graph_steps = max(1, cfg.graph_steps)
        self._graphs: Dict[int, torch.cuda.CUDAGraph] = {}

    # ------------------------------------------------------------------ util
    def lr(self, step: Optional[int] = None) -> float:
        s = self.step if step is None else step
        return learning_rate(s, self.n_local, self.B, self.cfg.base_lr, self.cfg.lr_decay)

    def sync_optimizer_state(self) -> None:
        """Replicated optimizer state: nothing to gather, except over the xGMI
        communicator's two-phase sync, whose fused all-reduce + SGD keeps each
        rank's momentum segment only (csrc/xgmi_comm.h all_reduce_sgd); the
        push and pull syncs keep the momentum replicated."""
        if self._syncs_over_xgmi() and self.xgmi_mode == "two-phase":
            self._sync.gather_segments(ptr(self.mom), self.layout.total, stream_handle())
            torch.cuda.synchronize(self.device)

    def _syncs_over_xgmi(self) -> bool:
        return self.xcomm is not None and self._sync is self.xcomm.native_handle

    @property
    def xgmi_mode(self) -> str:
        """The sync over the xGMI communicator: two-phase | push | pull."""
        m = self.exe.xgmi_mode if getattr(self, "exe", None) is not None else 0
        return XGMI_MODES[m]

    @property
    def sync_schedule(self) -> str:
        if not self.grad_sync:
            return "none"
        if self._syncs_over_xgmi():
            return {"two-phase": "xgmi", "push": "xgmi-push", "pull": "xgmi-pull"}[self.xgmi_mode]
        return "all-reduce"

    def extra_state(self):
        return {}

    def set_step(self, step: int) -> None:
        self.step = int(step)
        self.step_dev.fill_(int(step))

    def loss_value(self) -> float:
        return float(self.loss_rows.mean().item())

    def param_views(self):
        return self.layout.views(self.params)

    # ------------------------------------------------------------------ step
    def _launch_one(self) -> None:
        self.exe.train_step(stream_handle(), self._sync)

    def _set_sync(self, c, mode: Optional[str] = None) -> None:
        mode = self.xgmi_mode if mode is None else mode
        if c is self._sync and mode == self.xgmi_mode:
            return
        self.sync_optimizer_state()  # (two-phase xGMI: the sharded momentum made whole)
        self._sync = c
        self.exe.set_xgmi_mode(XGMI_MODE_IDS[mode])

    def _graph(self, n: int):
        key = (id(self._sync), self.xgmi_mode, n)
        g = self._graphs.get(key)
        if g is None:
            g = torch.cuda.CUDAGraph()
            try:
                with torch.cuda.graph(g):
                    for _ in range(n):
                        self._launch_one()
            except RuntimeError as e:  # keep training eagerly rather than fail the run
                print(f"[rank {self.rank}] hipGraph capture failed ({e}); using eager launches",
                      flush=True)
                self.use_graph = False
                torch.cuda.synchronize(self.device)
                return None
            self._graphs[key] = g
        return g

    def tune_schedule(self) -> int:
        """With an xGMI candidate next to RCCL (setup_comms): times TUNE
        replays of each sync's captured G-step graph and keeps the faster.
        The xGMI sync must first pass the health vote (no barrier timed out,
        identical replicas) and one trial step equal to RCCL's within
        XGMI_STEP_RTOL of the update (identical replicas cannot show a
        wrong-but-consistent sum).  Side-effect free (params, momentum and the
        device step are restored); collective (max-over-ranks times, voted
        checks).  Returns the trial steps run."""
        if self._tuned:
            return 0
        from ..parallel import dist as D
        from ..parallel.sync import replicas_identical
        from .mnist_engine import TUNE_REPLAYS, XGMI_STEP_RTOL
        G = self.graph_steps
        snap = (self.params.clone(), self.mom.clone(), self.step_dev.clone())
        xh = self.xcomm.native_handle
        cands = [("all-reduce", self._native_comm, "two-phase"), ("xgmi", xh, "two-phase"),
                 ("xgmi-push", xh, "push"), ("xgmi-pull", xh, "pull")]
        best, steps = None, 0

        def restore():
            self.params.copy_(snap[0])
            self.mom.copy_(snap[1])
            self.step_dev.copy_(snap[2])
            torch.cuda.synchronize(self.device)

        for name, c, mode in cands:
            if c is not self._native_comm and self.xcomm is None:
                self.tune_log[name] = None  # (the xGMI communicator timed out before)
                continue
            self._set_sync(c, mode)
            restore()
            g = self._graph(G)
            if D.allreduce_max_host(0.0 if g is not None else 1.0) != 0.0:
                self.tune_log[name] = None
                continue
            g.replay()
            torch.cuda.synchronize(self.device)
            steps += G
            if c is not self._native_comm:
                why = None
                if D.allreduce_max_host(float(self.xcomm.error())) != 0.0:
                    why = "a peer barrier timed out"
                else:
                    self.sync_optimizer_state()
                    if not (replicas_identical(self.params) and replicas_identical(self.mom)):
                        why = "the replicas differ after the trial steps"
                if why is None and not self.xcomm.emulated_comm:  # one eager step each
                    outs = []
                    for cc, pp in ((c, mode), (self._native_comm, "two-phase")):
                        self._set_sync(cc, pp)
                        restore()
                        self._launch_one()
                        torch.cuda.synchronize(self.device)
                        outs.append(self.params.clone())
                    self._set_sync(c, mode)
                    dx, ds = outs[0] - snap[0], outs[1] - snap[0]
                    ref = float(ds.abs().max())
                    err = float((dx - ds).abs().max())
                    worst = D.allreduce_max_host(err / max(ref, 1e-30))
                    bad = not (err <= XGMI_STEP_RTOL * ref)
                    if D.allreduce_max_host(1.0 if bad else 0.0) != 0.0:
                        why = (f"one trial step differs from the all-reduce's by {worst:.2e} of "
                               f"the largest update (bound {XGMI_STEP_RTOL:g})")
                    else:
                        self.xgmi_step_check[name] = worst
                if why is not None:
                    self.tune_log[name] = None
                    self.tune_reject[name] = why
                    if self.rank == 0:
                        print(f"[rank 0] sync {name} rejected: {why}", flush=True)
                    if "timed out" in why:
                        self.xcomm = None  # never used again (its barriers stop waiting)
                    continue
                restore()
            t0 = torch.cuda.Event(enable_timing=True)
            t1 = torch.cuda.Event(enable_timing=True)
            t0.record()
            for _ in range(TUNE_REPLAYS):
                g.replay()
            t1.record()
            torch.cuda.synchronize(self.device)
            steps += TUNE_REPLAYS * G
            us = D.allreduce_max_host(1000.0 * t0.elapsed_time(t1) / (TUNE_REPLAYS * G))
            self.tune_log[name] = round(us, 2)
            if best is None or us < best[0]:
                best = (us, c, mode)
        if best is None:
            best = (0.0, self._native_comm, "two-phase")
        self._set_sync(best[1], best[2])
        restore()
        self._tuned = True
        return steps

    def capture(self, k: int) -> None:
        if self.use_graph and k > 0:
            G = self.graph_steps
            if k >= G:
                self._graph(G)
            if k % G:
                self._graph(k % G)

    def train(self, k: int) -> None:
        if k <= 0:
            return
        if not self._tuned:  # side-effect free: restores the state it trained
            self.tune_schedule()
        done = 0
        if self.use_graph:
            G = self.graph_steps
            full, rem = divmod(k, G)
            g = self._graph(G) if full else None
            if g is not None:
                for _ in range(full):
                    g.replay()
                done = full * G
            if rem and self.use_graph:
                g = self._graph(rem)
                if g is not None:
                    g.replay()
                    done += rem
        for _ in range(k - done):
            self._launch_one()
        self.step += k

    def forward_backward_only(self) -> None:
        """Forward + backward, weight grads into the flat grad buffer (no
        sync, no SGD, no step increment): numerics tests."""
        self.exe.forward_backward(stream_handle())

    # ------------------------------------------------------------------ eval
    @torch.no_grad()
    def evaluate(self, x: np.ndarray, y: np.ndarray, chunk: int = 4096, dropout: bool = False,
                 return_logits: bool = False):
        n = int(x.shape[0])
        xd = self._eval_x.get(x, self.device)
        yd = torch.from_numpy(np.asarray(y).astype(np.int32)).to(self.device)
        errors = torch.zeros(1, dtype=torch.int32, device=self.device)
        logits = torch.empty(n, 10, device=self.device) if return_logits else None
        s = stream_handle()
        for a in range(0, n, chunk):
            m = min(chunk, n - a)
            lg = ptr(logits) + 4 * 10 * a if logits is not None else 0
            self._C.LenetExecutor.eval_chunk(self.ptrs, ptr(xd) + 4 * 3072 * a, ptr(yd) + 4 * a, m,
                                             lg, ptr(errors), s)
        err = 100.0 * float(errors.item()) / max(1, n)
        return (err, logits) if return_logits else err
