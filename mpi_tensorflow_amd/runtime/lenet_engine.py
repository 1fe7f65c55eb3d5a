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
from ..parallel.comm import DeviceComm
from ..utils.devcache import DeviceArrayCache
from ..utils.schedule import learning_rate

_OFFSETS = (("c1w", "c1_w"), ("c1b", "c1_b"), ("c2w", "c2_w"), ("c2b", "c2_b"), ("f1w", "f1_w"),
            ("f1b", "f1_b"), ("f2w", "f2_w"), ("f2b", "f2_b"), ("f3w", "f3_w"), ("f3b", "f3_b"))


class NativeLenetEngine:
    kind = "native-lenet5"

    def __init__(self, cfg: C.TrainConfig, train_x: np.ndarray, train_y: np.ndarray,
                 device: torch.device, rank: int = 0, world: int = 1,
                 comm: Optional[DeviceComm] = None, force_sync: bool = False):
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
        self.ptrs = p
        self.exe = C_.LenetExecutor(p)
        self._native_comm = None
        if self.grad_sync:
            self._native_comm = comm.native_handle
            if self._native_comm is None:
                raise RuntimeError("GPU grad sync needs the native RCCL communicator")
            if getattr(comm, "kind", "") == "host-staged":  # test comm: eager only
                comm.bases = [self.grads] + ([self.gb16] if self.gb16 is not None else [])
            self._xgmi = hasattr(comm, "register")
            if self._xgmi:  # xGMI peer to peer: peers read the grads and params,
                # and (to make it whole) the sharded momentum
                if self.gb16 is not None:
                    raise ValueError("the xGMI communicator reduces fp32 grads only")
                comm.register(self.grads, self.params, self.mom)
            # connection setup of the collective, outside any capture
            self._native_comm.all_reduce(ptr(self.grads), ptr(self.grads), self.layout.total, 7, 0,
                                         stream_handle())
            torch.cuda.synchronize(dev)
        self.use_graph = cfg.graph and getattr(comm, "kind", "") != "host-staged"
        self.graph_steps = max(1, cfg.graph_steps)
        self._graphs: Dict[int, torch.cuda.CUDAGraph] = {}

    # ------------------------------------------------------------------ util
    def lr(self, step: Optional[int] = None) -> float:
        s = self.step if step is None else step
        return learning_rate(s, self.n_local, self.B, self.cfg.base_lr, self.cfg.lr_decay)

    def sync_optimizer_state(self) -> None:
        """Replicated optimizer state: nothing to gather, except over the xGMI
        communicator, whose fused all-reduce + SGD keeps each rank's momentum
        segment only (csrc/xgmi_comm.h all_reduce_sgd)."""
        if self.grad_sync and getattr(self, "_xgmi", False):
            self._native_comm.gather_segments(ptr(self.mom), self.layout.total, stream_handle())
            torch.cuda.synchronize(self.device)

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
        self.exe.train_step(stream_handle(), self._native_comm)

    def _graph(self, n: int):
        g = self._graphs.get(n)
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
            self._graphs[n] = g
        return g

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
