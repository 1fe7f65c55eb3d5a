"""Training-step engines for the MNIST CNN.

Both engines own the same state - flat fp32 param / grad / momentum buffers
(`parallel/flat.py` layout), a step counter and the rank's device-resident
shard - and implement the same step semantics (reference `Cnn.run_process`
body, `/root/reference/mpipy.py:79-85`, + optimizer `:59-66`):

    offset = (step * B) % (N_local - B)                 (mpipy.py:80)
    forward on train[offset:offset+B] with dropout      (mpipy.py:155-167)
    grads of mean xent; SGD adds 5e-4*w on FC params    (mpipy.py:54-58)
    [grad all-reduce / world size]                      (DP)
    acc = 0.9 acc + g;  w -= lr(step) * acc;  step += 1 (mpipy.py:59-66)

* `NativeMnistEngine` (GPU): the fused gfx950 HIP kernels driven by the C++
  executor (`csrc/mnist_executor.cpp`); batch offset, dropout stream and LR
  are computed on the device from the device step counter, so G steps are
  captured ONCE into a hipGraph (torch.cuda.CUDAGraph) and replayed - no
  per-step host work, no H2D copies (the dataset is device resident).
* `TorchMnistEngine`: the plain-PyTorch fp32 oracle (CPU/gloo config 1 and
  the numerics reference for the kernels); it draws the identical dropout
  mask from utils/rng.py.
"""

from __future__ import annotations

import math
from typing import Dict, Optional

import numpy as np
import torch

from .. import config as C
from ..models import mnist_cnn as M
from ..ops import native, ptr, stream_handle
from ..parallel.comm import DeviceComm, XgmiDeviceComm, all_reduce_grads_
from ..utils import rng
from ..utils.data import batch_offset
from ..utils.schedule import learning_rate

# sync_schedule="auto": the single-communicator gradient-sync schedules
# (buckets / serial / sharded / factors, defer (fp32), csrc/mnist_executor.h) are timed on real
# training steps and the fastest is kept; all ranks take
# the decision from the same (max-over-ranks) timings.  The two-communicator
# "split" schedule (fastest against the comm-emulated 8-rank ring,
# docs/PERF_NOTES.md) issues collectives on two RCCL communicators from two
# streams at once; it is opt-in (--sync-schedule split) and never picked by
# auto until it has run on a real multi-GPU node.
TUNE_REPLAYS = 2
# _xgmi_step_matches: max |update(xGMI) - update(serial)| / max |update(serial)|
XGMI_STEP_RTOL = 1e-4


class MnistEngineBase:
    def __init__(self, cfg: C.TrainConfig, train_x: np.ndarray, train_y: np.ndarray,
                 device: torch.device, rank: int = 0, world: int = 1,
                 comm: Optional[DeviceComm] = None):
        self.cfg = cfg
        self.device = device
        self.rank, self.world = rank, world
        self.comm = comm
        self.layout = M.layout()
        self.B = cfg.batch_size
        self.n_local = int(train_x.shape[0])
        if self.n_local <= self.B:
            raise ValueError(f"local shard of {self.n_local} rows must exceed batch {self.B}")
        self.params = torch.zeros(self.layout.total, dtype=torch.float32, device=device)
        self.grads = torch.zeros_like(self.params)
        self.mom = torch.zeros_like(self.params)
        host = torch.zeros(self.layout.total, dtype=torch.float32)
        M.init_params(host, self.layout, seed=cfg.seed)
        self.params.copy_(host)
        self.step = 0  # host mirror of the global step (TF iter_)
        self.drop_seed = cfg.seed
        self.drop_rank = 0 if cfg.same_seed_all_ranks else rank  # quirk Q14
        self.grad_sync = cfg.sync == "grad" and world > 1 and comm is not None

    # views -----------------------------------------------------------------
    def param_views(self) -> Dict[str, torch.Tensor]:
        return self.layout.views(self.params)

    def lr(self, step: Optional[int] = None) -> float:
        s = self.step if step is None else step
        return learning_rate(s, self.n_local, self.B, self.cfg.base_lr, self.cfg.lr_decay)

    def l2_value(self) -> float:
        p = self.param_views()
        return float(self.cfg.l2 * M.l2_term(p).item())

    def state_tensors(self):
        return self.params, self.mom

    def sync_optimizer_state(self) -> None:
        """Makes `mom` whole on every rank (a sharded optimizer keeps only
        its own shard current); no-op for replicated optimizers."""

    def extra_state(self):
        """Non-trained state saved with checkpoints (none for this model)."""
        return {}

    def set_step(self, step: int) -> None:
        self.step = int(step)

    def synchronize(self) -> None:
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)


class TorchMnistEngine(MnistEngineBase):
    """fp32 PyTorch oracle engine (CPU or GPU)."""

    kind = "torch"

    def __init__(self, cfg, train_x, train_y, device, rank=0, world=1, comm=None):
        super().__init__(cfg, train_x, train_y, device, rank, world, comm)
        self.train_x = torch.from_numpy(np.ascontiguousarray(train_x, np.float32)).to(device)
        self.train_y = torch.from_numpy(np.asarray(train_y).astype(np.int64)).to(device)
        self.last_loss = float("nan")

    def dropout_mask(self, step: int, rows: int, salt: int = 0) -> torch.Tensor:
        key = rng.dropout_key(self.drop_seed, self.drop_rank, step, salt)
        return rng.keep_mask_torch(key, (rows, M.FC1_OUT), self.cfg.dropout_keep, self.device)

    def forward_backward(self, step: int):
        off = batch_offset(step, self.n_local, self.B)
        x = self.train_x[off:off + self.B]
        y = self.train_y[off:off + self.B]
        views = {k: v.detach().clone().requires_grad_(True) for k, v in self.param_views().items()}
        logits = M.forward(views, x, self.dropout_mask(step, self.B), self.cfg.dropout_keep)
        data_loss = torch.nn.functional.cross_entropy(logits, y)
        grads = torch.autograd.grad(data_loss, [views[s.name] for s in self.layout.specs])
        gv = self.layout.views(self.grads)
        for s, g in zip(self.layout.specs, grads):
            gv[s.name].copy_(g)
        self.last_loss = float(data_loss.item())
        return data_loss

    def train(self, k: int) -> None:
        for _ in range(k):
            self.forward_backward(self.step)
            gscale = 1.0
            if self.grad_sync:
                all_reduce_grads_(self.comm, self.grads, self.cfg.grad_comm_dtype)
                gscale = 1.0 / self.world
            lr = self.lr(self.step)
            _, l2_end = self.layout.l2_range()
            g = self.grads * gscale
            g[:l2_end] += self.cfg.l2 * self.params[:l2_end]
            self.mom.mul_(self.cfg.momentum).add_(g)
            self.params.sub_(lr * self.mom)
            self.step += 1

    def loss_value(self) -> float:
        return self.last_loss + self.l2_value()

    @torch.no_grad()
    def evaluate(self, x: np.ndarray, y: np.ndarray, chunk: int = 2000, dropout: bool = False,
                 return_logits: bool = False):
        views = self.param_views()
        wrong = 0
        outs = []
        for a in range(0, x.shape[0], chunk):
            xb = torch.from_numpy(x[a:a + chunk]).to(self.device)
            mask = None
            if dropout:
                mask = self.dropout_mask(self.step, xb.shape[0], rng.EVAL_SALT)
            lg = M.forward(views, xb, mask, self.cfg.dropout_keep)
            if return_logits:
                outs.append(lg)
            pred = lg.argmax(1).cpu().numpy()
            wrong += int((pred != y[a:a + chunk]).sum())
        err = 100.0 * wrong / max(1, x.shape[0])
        if return_logits:
            return err, (torch.cat(outs) if outs else torch.empty(0, 10, device=self.device))
        return err


class NativeMnistEngine(MnistEngineBase):
    """fused HIP kernels + C++ executor + hipGraph replay (MI355X); fp32
    (v_mfma_f32_32x32x2_f32) or bf16 (v_mfma_f32_32x32x16_bf16, fp32 master
    weights / grads / momentum) per cfg.dtype."""

    kind = "native"

    def __init__(self, cfg, train_x, train_y, device, rank=0, world=1, comm=None,
                 force_sync: bool = False, fc1_feature_major: bool = False,
                 xcomm: Optional[XgmiDeviceComm] = None):
        """fc1_feature_major (labs): the fp32 Winograd step's conv2 forward
        also writes a2 feature-major and the fc1 forward reads its operands
        straight from L2 (fc1_fwd_t_kernel) instead of staging them through
        LDS.  Equal in isolation (8.0 vs 8.3 us), but 3 us SLOWER in the step
        (10.0 vs 6.9 us: the 4-byte scattered a2t stores of 256 blocks leave
        partial lines in every XCD's L2), so off (docs/PERF_NOTES.md)."""
        super().__init__(cfg, train_x, train_y, device, rank, world, comm)
        if force_sync and comm is not None:  # exercise the collective path at world 1
            self.grad_sync = True
        if device.type != "cuda":
            raise RuntimeError("NativeMnistEngine needs a GPU")
        if self.B % 32 != 0:
            raise ValueError("native MNIST engine needs a batch size that is a multiple of 32")
        C_ = native()
        self._C = C_
        dev = device
        B = self.B
        f32 = dict(dtype=torch.float32, device=dev)
        u8 = dict(dtype=torch.uint8, device=dev)
        self.train_x = torch.from_numpy(np.ascontiguousarray(train_x, np.float32)).to(dev)
        self.train_y = torch.from_numpy(np.ascontiguousarray(train_y).astype(np.int32)).to(dev)
        assert self.train_x.shape[1:] == (28, 28, 1)
        self.step_dev = torch.zeros(1, dtype=torch.int64, device=dev)
        self.lr_dev = torch.zeros(1, **f32)
        self.correct_dev = torch.zeros(1, dtype=torch.int32, device=dev)
        k = C_.mnist
        self.bufs = dict(
            a1=torch.empty(B * 14 * 14 * 32, **f32), idx1=torch.empty(B * 14 * 14 * 32, **u8),
            a2=torch.empty(B * M.FC1_IN, **f32), idx2=torch.empty(B * M.FC1_IN, **u8),
            fc1_part=torch.empty(k.fc1_part_floats(B), **f32),
            hd=torch.empty(B * M.FC1_OUT, **f32), dh=torch.empty(B * M.FC1_OUT, **f32),
            dlog=torch.empty(B * 10, **f32), loss_rows=torch.zeros(B, **f32),
            dy2=torch.empty(B * 14 * 14 * 64, **f32), da1m=torch.empty(B * 14 * 14 * 32, **f32),
            # channel-major dY2 with a zero border that is never written
            dy2t=torch.zeros(B * 64 * 18 * 20, **f32),
            part2=torch.empty(k.part2_floats(B), **f32), part1=torch.empty(k.part1_floats(B), **f32),
            w2t=torch.empty(25 * 64 * 32, **f32),
            # zero-bordered NHWC a1 (filter-grad operand; the border is never written)
            a1pf=torch.zeros(B * 18 * 18 * 32, **f32),
        )
        self.bf16 = cfg.dtype == "bf16"
        self.wino = (not self.bf16) and cfg.conv_algo == "winograd"
        if self.wino:  # Winograd-transformed conv2 filters (csrc/kernels/wino.h)
            self.bufs.update(wino_u=torch.empty(36 * 32 * 64, **f32),
                             wino_ud=torch.empty(36 * 64 * 32, **f32),
                             # the filter gradient's point slabs replace the 25-tap ones
                             part2=torch.empty(k.part2_floats_wino(B), **f32))
            if fc1_feature_major:  # a2 feature-major, the fc1 forward's direct operand
                self.bufs["a2ft"] = torch.empty(M.FC1_IN * B, **f32)
        self.fac = None
        hcomm = comm.native_handle if (self.grad_sync and comm is not None) else None
        nfac = hcomm.size if hcomm is not None else 1
        self.comm_is_xgmi = isinstance(comm, XgmiDeviceComm)
        if nfac > 1 and not self.bf16:
            # SCHED_FACTORS / SCHED_XGMI_FAC: rank-major gathered FC factors;
            # this rank's forward / head kernels write their slot in place
            # (csrc/mnist_executor.cpp train_step_factors, train_step_xgmi_fac).  Sized by the communicator (an emulated
            # N-rank comm on one GPU gets N slots, rank 0's filled).
            crank = hcomm.rank
            self.fac = dict(a2=torch.zeros(nfac * B * M.FC1_IN, **f32),
                            dh=torch.zeros(nfac * B * M.FC1_OUT, **f32),
                            hd=torch.zeros(nfac * B * M.FC1_OUT, **f32),
                            dlog=torch.zeros(nfac * B * 10, **f32))
            for name, t in self.fac.items():
                n = t.numel() // nfac
                self.bufs[name] = t[crank * n:(crank + 1) * n]
        if self.bf16:
            # bf16 activation images (zero borders are never written) and
            # weight shadows; layouts in csrc/kernels/mnist_bf16.h
            b16 = dict(dtype=torch.bfloat16, device=dev)
            self.bufs.update(
                a1p=torch.zeros(B * 18 * 18 * 32, **b16), a1t=torch.zeros(B * 32 * 18 * 24, **b16),
                a2h=torch.zeros(B * M.FC1_IN, **b16), a2t=torch.zeros(M.FC1_IN * B, **b16),
                dy2p=torch.zeros(B * 18 * 18 * 64, **b16), dy2t=torch.zeros(B * 64 * 14 * 16, **b16),
                dh16=torch.zeros(B * M.FC1_OUT, **b16), dht16=torch.zeros(M.FC1_OUT * B, **b16),
                w1b=torch.zeros(M.FC1_IN * M.FC1_OUT, **b16),
                w1t=torch.zeros(M.FC1_OUT * M.FC1_IN, **b16),
                w2tb=torch.zeros(25 * 64 * 32, **b16), w2b=torch.zeros(25 * 32 * 64, **b16),
                part2=torch.empty(k.part2_floats_bf16(B), **f32),
            )
            for name in ("a1", "a2", "dy2", "w2t", "a1pf"):  # fp32-only buffers
                self.bufs[name] = torch.empty(0, **f32)
        p = C_.MnistPtrs()
        p.train_x, p.train_y = ptr(self.train_x), ptr(self.train_y)
        p.n_local, p.batch = self.n_local, B
        p.params, p.grads, p.mom = ptr(self.params), ptr(self.grads), ptr(self.mom)
        lay = self.layout
        p.total = lay.total
        p.l2_end = lay.l2_range()[1]
        p.bucket1 = lay.buckets()[0][1]
        for attr, name in (("off_w4", "fc2_weight"), ("off_b4", "fc2_bias"), ("off_w3", "fc1_weight"),
                           ("off_b3", "fc1_bias"), ("off_w2", "conv2_weight"), ("off_b2", "conv2_bias"),
                           ("off_w1", "conv1_weight"), ("off_b1", "conv1_bias")):
            setattr(p, attr, lay.offsets[name])
        p.step, p.lr, p.correct = ptr(self.step_dev), ptr(self.lr_dev), ptr(self.correct_dev)
        for name, t in self.bufs.items():
            setattr(p, name, ptr(t))
        p.keep_prob, p.base_lr, p.lr_decay = cfg.dropout_keep, cfg.base_lr, cfg.lr_decay
        p.l2, p.momentum = cfg.l2, cfg.momentum
        p.seed, p.rank, p.world = cfg.seed, self.drop_rank, world
        p.bf16 = 1 if self.bf16 else 0
        p.wino = 1 if self.wino else 0
        self.gb16 = None  # bf16 gradient wire staging (--grad-comm-dtype bf16)
        if cfg.grad_comm_dtype == "bf16" and world > 1:
            self.gb16 = torch.zeros(self.layout.total, dtype=torch.bfloat16, device=dev)
            p.grad_bf16, p.gb16 = 1, ptr(self.gb16)
        if self.fac is not None:
            p.a2_all, p.dh_all = ptr(self.fac["a2"]), ptr(self.fac["dh"])
            p.hd_all, p.dlog_all = ptr(self.fac["hd"]), ptr(self.fac["dlog"])
            p.fac_ranks = nfac
        self.ptrs = p
        self.exe = C_.MnistExecutor(p)
        # xGMI peer-to-peer schedule: the peers read this rank's grads / params
        # (and, to gather the sharded FC momentum, its momentum) directly
        self.xcomm = comm if self.comm_is_xgmi else xcomm
        if not self.grad_sync:
            self.xcomm = None
        if self.xcomm is not None:
            # + the conv-grad exchange buffer of the step launch (two halves
            # by barrier epoch parity: no closing barrier for the conv blocks)
            cf = C_.mnist.xgmi_conv_floats(self.layout.offsets["conv1_bias"])
            self.xconv = torch.zeros(2 * cf, device=dev)
            facs = list(self.fac.values()) if self.fac is not None else []
            if facs and self.xcomm.size != nfac:
                facs = []  # sized for another communicator: no xgmi-fac
            self.xcomm.register(self.grads, self.params, self.mom, self.xconv, *facs)
            self.exe.set_xgmi(self.xcomm.native_handle)
            self.exe.set_xgmi_xconv(ptr(self.xconv))
        self.comm_stream = torch.cuda.Stream(device=dev) if self.grad_sync else None
        self._native_comm = self.comm.native_handle if (self.grad_sync and self.comm) else None
        if self.grad_sync and self._native_comm is None:
            raise RuntimeError("grad sync on the native engine needs the native RCCL communicator")
        self.comm2 = None  # second communicator (split schedule: conv bucket on the compute stream)
        if self.grad_sync and cfg.sync_schedule == "split":
            self.comm2 = self.comm.duplicate()
        self._native_comm2 = self.comm2.native_handle if self.comm2 is not None else None
        if self.grad_sync:
            self.exe.set_defer_split(float(cfg.defer_split))
            self.exe.set_schedule(self._pick_schedule(cfg.sync_schedule, self._native_comm.size))
        if getattr(self.comm, "kind", "") == "host-staged":  # test comm: eager only
            self.comm.bases = [self.grads, self.params, self.mom] + (
                [self.gb16] if self.gb16 is not None else []) + (
                list(self.fac.values()) if self.fac is not None else [])
        self._graphs: Dict[tuple, torch.cuda.CUDAGraph] = {}
        self._derived_ver = None  # params version the derived weights were made from
        self.use_graph = cfg.graph and getattr(self.comm, "kind", "") != "host-staged"
        self.graph_steps = max(1, cfg.graph_steps)
        # (auto always has >= 2 candidates: buckets and serial)
        self._tuned = not (self.grad_sync and cfg.sync_schedule == "auto" and self.use_graph)
        self.tune_log: Dict[str, float] = {}
        self.tune_reject: Dict[str, str] = {}  # candidate -> why it was dropped
        self.xgmi_step_check: Dict[str, float] = {}  # xGMI schedule -> measured update rel. diff
        self.tune_steps_run = 0
        self._eval_ws = None
        if self.grad_sync:  # connection setup of every collective used, outside any capture
            c, g, n, hs = self._native_comm, ptr(self.grads), lay.total, stream_handle()
            c.all_reduce(g, g, n, 7, 0, hs)
            if self.exe.sharded_ok(c.size) and not self.comm_is_xgmi:  # grads are zero: RS / AG leave them zero
                chunk = self.ptrs.bucket1 // c.size
                c.reduce_scatter(g, g + 4 * chunk * c.rank, chunk, 7, 0, hs)
                c.all_gather(g + 4 * chunk * c.rank, g, chunk, 7, hs)
            if self.exe.factors_ok(c.size) and not self.comm_is_xgmi:  # factor all-gathers, in place
                for t in self.fac.values():
                    k = t.numel() // c.size
                    c.all_gather(ptr(t) + 4 * k * c.rank, ptr(t), k, 7, hs)
            if self._native_comm2 is not None:
                self._native_comm2.all_reduce(g, g, n, 7, 0, hs)
            torch.cuda.synchronize(dev)

    def set_step(self, step: int) -> None:
        super().set_step(step)
        self.step_dev.fill_(int(step))

    def _pick_schedule(self, name: str, nranks: int) -> int:
        E = self._C.MnistExecutor
        if name == "buckets":
            return E.SCHED_BUCKETS
        if name == "sharded" and self.exe.sharded_ok(nranks):
            return E.SCHED_SHARDED_FC
        if name == "split" and self._native_comm2 is not None:
            return E.SCHED_SPLIT
        if name == "factors" and self.exe.factors_ok(nranks) and not self.comm_is_xgmi:
            return E.SCHED_FACTORS
        if name == "serial":
            return E.SCHED_SERIAL
        if name == "defer" and self.exe.defer_ok():
            return E.SCHED_DEFER
        if name == "xgmi-step" and self.exe.xgmi_ok():
            return E.SCHED_XGMI_STEP
        if name == "xgmi-fac" and self.exe.xgmi_fac_ok():
            return E.SCHED_XGMI_FAC
        if (name == "xgmi" or self.comm_is_xgmi) and self.exe.xgmi_ok():
            return E.SCHED_XGMI
        if self.comm_is_xgmi:
            return E.SCHED_SERIAL  # (the xGMI comm's all-reduce)
        return E.SCHED_BUCKETS  # "auto" until tuned

    def _set_schedule(self, sched: int) -> None:
        """Switches the executor's sync schedule.  Leaving the sharded FC
        schedule first all-gathers the FC momentum (each rank only kept its own
        1/N shard current), otherwise the replicas would continue with
        different momenta on the shards they do not own and diverge."""
        if sched == self.exe.schedule:
            return
        self.sync_optimizer_state()
        self.exe.set_schedule(sched)

    @property
    def sync_schedule(self) -> str:
        if not self.grad_sync:
            return "none"
        E = self._C.MnistExecutor
        return {E.SCHED_SHARDED_FC: "sharded", E.SCHED_SPLIT: "split",
                E.SCHED_FACTORS: "factors", E.SCHED_SERIAL: "serial",
                E.SCHED_DEFER: "defer", E.SCHED_XGMI: "xgmi",
                E.SCHED_XGMI_STEP: "xgmi-step", E.SCHED_XGMI_FAC: "xgmi-fac"}.get(
                    self.exe.schedule,
                                                                           "buckets")

    def sync_optimizer_state(self) -> None:
        if self.grad_sync:
            self.exe.gather_optimizer_state(stream_handle(), self._native_comm,
                                            stream_handle(self.comm_stream))

    # --------------------------------------------------------------- steps
    def _launch_one(self):
        cs = stream_handle(self.comm_stream) if self.comm_stream is not None else 0
        self.exe.train_step(stream_handle(), self._native_comm, cs, self._native_comm2)

    def _graph(self, n: int, sticky: bool = True) -> Optional[torch.cuda.CUDAGraph]:
        """Captured graph of n steps under the current schedule.  A failed
        capture switches the engine to eager launches (sticky) or, while the
        schedules are being tuned, only drops that candidate."""
        key = (self.exe.schedule, n)
        g = self._graphs.get(key)
        if g is None:
            if self.comm_stream is not None:
                self.comm_stream.wait_stream(torch.cuda.current_stream())
            g = torch.cuda.CUDAGraph()
            try:
                with torch.cuda.graph(g):
                    for _ in range(n):
                        self._launch_one()
                    self.exe.join(stream_handle())  # comm stream rejoins inside the capture
            except RuntimeError as e:
                # e.g. a collective library build that cannot be captured:
                # keep training with eager launches instead of failing the run
                print(f"[rank {self.rank}] hipGraph capture failed ({e}); "
                      + ("using eager launches" if sticky else "skipping this schedule"),
                      flush=True)
                self.use_graph = self.use_graph and not sticky
                torch.cuda.synchronize(self.device)
                return None
            # the executable goes to the device now, not inside its first
            # (possibly timed) launch
            self._C.graph_upload(g.raw_cuda_graph_exec(), stream_handle())
            self._graphs[key] = g
        return g

    def _tune_candidates(self):
        E = self._C.MnistExecutor
        n = self._native_comm.size
        xg = []
        if self.exe.xgmi_ok():  # fp32: the FC exchange in the conv2 backward, or in the step launch
            xg = [(E.SCHED_XGMI, "xgmi")] + ([] if self.bf16 else [(E.SCHED_XGMI_STEP, "xgmi-step")])
        # the FC gradients from the gathered factors (another summation order:
        # under --deterministic auto keeps to the bit-identical schedules)
        if self.exe.xgmi_fac_ok() and not self.cfg.deterministic:
            xg.append((E.SCHED_XGMI_FAC, "xgmi-fac"))
        if self.comm_is_xgmi:  # no comm stream: the fused launches or the plain all-reduce
            return xg + [(E.SCHED_SERIAL, "serial")]
        cands = [(E.SCHED_BUCKETS, "buckets"), (E.SCHED_SERIAL, "serial")]
        cands += xg
        if self.exe.sharded_ok(n):
            cands.append((E.SCHED_SHARDED_FC, "sharded"))
        # the factor schedule forms the FC gradients in another summation
        # order: under --deterministic auto keeps to the bit-identical ones
        if self.exe.factors_ok(n) and not self.cfg.deterministic:
            cands.append((E.SCHED_FACTORS, "factors"))
        if self.exe.defer_ok():
            cands.append((E.SCHED_DEFER, "defer"))
        return cands

    def tune_steps(self) -> int:
        """Training steps tune_schedule() runs (and then discards)."""
        if self._tuned:
            return 0
        return len(self._tune_candidates()) * (1 + TUNE_REPLAYS) * self.graph_steps

    def tune_schedule(self) -> int:
        """Times TUNE_REPLAYS graph replays of each sync schedule (after one
        untimed replay each) and keeps the fastest.  Side-effect free: the
        params, momentum and device step are snapshotted first and restored
        afterwards, so training continues exactly where it was (the trial
        steps do not count towards `step`).  Collective over the ranks: all
        ranks decide from the same max-over-ranks timings.  Returns the
        number of trial steps run."""
        if self._tuned:
            return 0
        from ..parallel import dist as D
        E = self._C.MnistExecutor
        G = self.graph_steps
        steps = 0
        best = None
        self.exe.join(stream_handle())
        # the candidates' steps take the derived weights (Winograd transforms,
        # bf16 shadows) as current: derive them from the weights first
        self.exe.refresh_shadows(stream_handle())
        snap = (self.params.clone(), self.mom.clone(), self.step_dev.clone())
        cands = self._tune_candidates()
        xgmi_scheds = (E.SCHED_XGMI, E.SCHED_XGMI_STEP, E.SCHED_XGMI_FAC)
        xgmi_dead = False
        for sched, name in cands:
            uses_xgmi = sched in xgmi_scheds or self.comm_is_xgmi
            if uses_xgmi and xgmi_dead:
                # a timed-out barrier leaves the communicator's sticky error set and
                # its later barriers no longer wait: nothing over it may run again
                self.tune_log[name] = None
                continue
            self._set_schedule(sched)
            g = self._graph(G, sticky=(sched == cands[-1][0] if self.comm_is_xgmi
                                       else sched == E.SCHED_BUCKETS))
            # the decision must be collective: a candidate any rank could not
            # capture is dropped on every rank
            ok = D.allreduce_max_host(0.0 if g is not None else 1.0) == 0.0
            if not ok:
                if sched == E.SCHED_BUCKETS:  # no graphs at all: keep buckets, eager
                    break
                self.tune_log[name] = None
                continue
            g.replay()
            torch.cuda.synchronize(self.device)
            if uses_xgmi:
                why = self._xgmi_healthy()
                if why is None and sched in xgmi_scheds:
                    why = self._xgmi_step_matches(sched, snap)
                if why is not None:
                    self.tune_log[name] = None  # never pick it
                    self.tune_reject[name] = why
                    if self.rank == 0:
                        print(f"[rank 0] sync schedule {name} rejected: {why}", flush=True)
                    if "timed out" in why:
                        xgmi_dead = True
                        if self.comm_is_xgmi:
                            raise RuntimeError(f"xGMI communicator failed during the sync-schedule "
                                               f"autotune ({why}); there is no other communicator")
                        # RCCL trains on; the dead xGMI comm leaves the health votes
                        self.xcomm = None
                    continue
            t0 = torch.cuda.Event(enable_timing=True)
            t1 = torch.cuda.Event(enable_timing=True)
            t0.record()
            for _ in range(TUNE_REPLAYS):
                g.replay()
            t1.record()
            torch.cuda.synchronize(self.device)
            steps += (1 + TUNE_REPLAYS) * G
            us = D.allreduce_max_host(1000.0 * t0.elapsed_time(t1) / (TUNE_REPLAYS * G))
            self.tune_log[name] = round(us, 2)
            if best is None or us < best[0]:
                best = (us, sched)
        if best is None and self.comm_is_xgmi:
            raise RuntimeError("no sync schedule over the xGMI communicator passed its checks: "
                               + "; ".join(f"{k}: {v}" for k, v in self.tune_reject.items()))
        self._set_schedule(best[1] if best is not None else E.SCHED_BUCKETS)
        self.exe.join(stream_handle())
        self.params.copy_(snap[0])
        self.mom.copy_(snap[1])
        self.step_dev.copy_(snap[2])
        torch.cuda.synchronize(self.device)
        self._tuned = True
        self.tune_steps_run = steps
        return steps

    def _xgmi_healthy(self) -> Optional[str]:
        """Collective: None when no rank's xGMI barrier timed out (the device
        kernels never hang: a missing peer sets a sticky error bit instead)
        and the replicas agree bit for bit after the trial steps, else why."""
        from ..parallel import dist as D
        from ..parallel.sync import replicas_identical
        bad = self.xcomm.error() if self.xcomm is not None else 0
        if D.allreduce_max_host(float(bad)) != 0.0:
            return "a peer barrier timed out"
        if self.xcomm is None or self.xcomm.emulated_comm:
            return None
        # replicas must agree bit for bit after the trial steps (a lost or torn
        # peer read would show here): gather the sharded momentum and compare
        self.sync_optimizer_state()
        torch.cuda.synchronize(self.device)
        if not (replicas_identical(self.params) and replicas_identical(self.mom)):
            return "the replicas differ after the trial steps"
        return None

    def _xgmi_step_matches(self, sched: int, snap) -> Optional[str]:
        """Collective: one eager step of the xGMI schedule `sched` against one
        eager step of the serial schedule over the other communicator (RCCL;
        the xGMI comm's exactness-checked all-reduce when it is the only one),
        both from the state `snap`.  Identical replicas cannot reveal a
        wrong-but-consistent reduction (every rank gathers the same wrong
        segments), this can: the two parameter updates must agree to
        XGMI_STEP_RTOL of the largest update (rank-order vs RCCL summation is
        ~1e-7; a rank left out of the sum is ~1/N).  None = match, else why.
        The state is restored to `snap` afterwards.  Emulated communicators
        are not compared (their numerics are not those of N ranks)."""
        from ..parallel import dist as D
        if self.xcomm is None or self.xcomm.emulated_comm:
            return None
        E = self._C.MnistExecutor
        s = stream_handle()
        outs = []
        for sc in (sched, E.SCHED_SERIAL):
            self._set_schedule(sc)
            self.params.copy_(snap[0])
            self.mom.copy_(snap[1])
            self.step_dev.copy_(snap[2])
            self.exe.refresh_shadows(s)
            self._launch_one()
            self.exe.join(s)
            torch.cuda.synchronize(self.device)
            outs.append(self.params.clone())
        self._set_schedule(sched)
        self.params.copy_(snap[0])
        self.mom.copy_(snap[1])
        self.step_dev.copy_(snap[2])
        self.exe.refresh_shadows(s)
        torch.cuda.synchronize(self.device)
        dx, ds = outs[0] - snap[0], outs[1] - snap[0]
        ref = float(ds.abs().max())
        err = float((dx - ds).abs().max())
        bad = not (err <= XGMI_STEP_RTOL * ref) or not math.isfinite(err)
        worst = D.allreduce_max_host(err / max(ref, 1e-30))
        if D.allreduce_max_host(1.0 if bad else 0.0) != 0.0:
            return (f"one trial step differs from the serial schedule's by {worst:.2e} of the "
                    f"largest update (bound {XGMI_STEP_RTOL:g})")
        self.xgmi_step_check[self.sync_schedule] = worst
        return None

    def prewarm_train(self, ms: float) -> float:
        """Untimed, side-effect-free training replays for ~`ms` of wall time
        (bench.py --prewarm train): the captured G-step graph is replayed
        with the params, momentum and device step snapshotted first and
        restored afterwards (as tune_schedule), so training continues
        exactly where it was.  The replay count is agreed over the ranks
        (max) before the loop: the graph holds the collectives at N > 1.
        Returns the wall time spent (ms)."""
        if ms <= 0 or not self.use_graph:
            return 0.0
        import time

        from ..parallel import dist as D
        if not self._tuned:
            self.tune_schedule()
        g = self._graph(self.graph_steps)
        if g is None:
            return 0.0
        t_start = time.perf_counter()
        self.exe.join(stream_handle())
        self.exe.refresh_shadows(stream_handle())
        snap = (self.params.clone(), self.mom.clone(), self.step_dev.clone())
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize(self.device)
        dt = max(time.perf_counter() - t0, 1e-6)
        reps = int(D.allreduce_max_host(float(max(1, math.ceil(ms / 1000.0 / dt)))))
        for _ in range(reps - 1):
            g.replay()
        self.exe.join(stream_handle())
        self.params.copy_(snap[0])
        self.mom.copy_(snap[1])
        self.step_dev.copy_(snap[2])
        torch.cuda.synchronize(self.device)
        return round(1000.0 * (time.perf_counter() - t_start), 1)

    def train(self, k: int) -> None:
        if k <= 0:
            return
        if not self._tuned:  # side-effect free: restores the state it trained
            self.tune_schedule()
        # the steps' SGD launches keep the derived weights (Winograd transforms,
        # bf16 shadows) current for the next step; they are re-derived from the
        # master weights only when something outside the steps changed those
        # (checkpoint load, parameter averaging, a tune's restore: every torch
        # in-place write bumps the tensor's version; the kernels' raw-pointer
        # writes do not).  Skipping the launch keeps it out of short timed runs.
        if self._derived_ver != self.params._version:
            self.exe.refresh_shadows(stream_handle())
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
        for _ in range(k - done):  # eager (no graphs, or capture unavailable)
            self._launch_one()
        self.exe.join(stream_handle())
        self.step += k
        self._derived_ver = self.params._version

    def capture(self, k: int) -> None:
        """Pre-captures the graphs `train(k)` will replay (outside timing)."""
        if self.use_graph:
            G = self.graph_steps
            if k >= G:
                self._graph(G)
            if k % G:
                self._graph(k % G)

    def forward_backward_only(self) -> None:
        """Forward + backward into the flat grad buffer; no sync, no SGD, no
        step increment (used by the numerics tests)."""
        self.exe.forward_backward(stream_handle())

    def loss_value(self) -> float:
        return float(self.bufs["loss_rows"].mean().item()) + self.l2_value()

    def device_lr(self) -> float:
        return float(self.lr_dev.item())

    # ---------------------------------------------------------------- eval
    @torch.no_grad()
    def evaluate(self, x: np.ndarray, y: np.ndarray, chunk: int = 2000, dropout: bool = False,
                 x_dev: Optional[torch.Tensor] = None, y_dev: Optional[torch.Tensor] = None,
                 return_logits: bool = False):
        dev = self.device
        if x_dev is None:
            x_dev = torch.from_numpy(np.ascontiguousarray(x, np.float32)).to(dev)
            y_dev = torch.from_numpy(np.ascontiguousarray(y).astype(np.int32)).to(dev)
        n = int(x_dev.shape[0])
        chunk = min(chunk, max(n, 1))
        if self._eval_ws is None or self._eval_ws[0] < chunk:
            f32 = dict(dtype=torch.float32, device=dev)
            if self.bf16:
                cp = (chunk + 7) // 8 * 8
                b16 = dict(dtype=torch.bfloat16, device=dev)
                self._eval_ws = (chunk, torch.zeros(cp * 18 * 18 * 32, **b16),
                                 torch.zeros(cp * M.FC1_IN, **b16),
                                 torch.empty(chunk * M.FC1_OUT, **f32))
            else:
                self._eval_ws = (chunk, torch.empty(chunk * 14 * 14 * 32, **f32),
                                 torch.empty(chunk * M.FC1_IN, **f32),
                                 torch.empty(chunk * M.FC1_OUT, **f32))
        _, a1, a2, h = self._eval_ws
        errors = torch.zeros(1, dtype=torch.int32, device=dev)
        logits = torch.empty(n, 10, dtype=torch.float32, device=dev) if return_logits else None
        keep = self.cfg.dropout_keep if dropout else 1.0
        key = rng.dropout_key(self.drop_seed, self.drop_rank, self.step, rng.EVAL_SALT)
        s = stream_handle()
        for a in range(0, n, chunk):
            m = min(chunk, n - a)
            lg = ptr(logits) + 4 * 10 * a if logits is not None else 0
            self._C.MnistExecutor.eval_chunk(self.ptrs, ptr(x_dev) + 4 * 784 * a, ptr(y_dev) + 4 * a,
                                             m, ptr(a1), ptr(a2), ptr(h), lg, ptr(errors), keep,
                                             key, s)
        err = 100.0 * float(errors.item()) / max(1, n)
        return (err, logits) if return_logits else err


def make_engine(cfg: C.TrainConfig, train_x, train_y, device: torch.device, rank=0, world=1,
                comm=None, backend: Optional[str] = None, force_sync: bool = False,
                xcomm: Optional[XgmiDeviceComm] = None):
    backend = backend or cfg.backend
    if backend == "auto":
        backend = "native" if device.type == "cuda" else "torch"
    if cfg.dtype != "fp32" and backend != "native":
        raise NotImplementedError(f"dtype {cfg.dtype} needs the native (GPU) MNIST engine")
    if backend == "native":
        return NativeMnistEngine(cfg, train_x, train_y, device, rank, world, comm, force_sync,
                                 xcomm=xcomm)
    return TorchMnistEngine(cfg, train_x, train_y, device, rank, world, comm)
