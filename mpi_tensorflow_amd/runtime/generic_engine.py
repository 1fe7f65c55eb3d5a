"""Training engine for the generic models (LeNet-5, ResNet-18).

Same contract as the MNIST engines (runtime/mnist_engine.py): flat fp32
param / grad / momentum buffers, the reference's LR schedule and momentum
SGD (/root/reference/mpipy.py:59-66), batch offset (step*B) % (N-B), DP by
per-step gradient all-reduce of the flat grad buffer.

With cfg.dtype == "bf16" the convolutions run their MFMAs on bf16 operands
(bf16 copies / twins of activations and output gradients, re-laid bf16
weights, csrc/kernels/conv_bf16.hip; fp32 accumulation).  A conv whose only
consumer is a BatchNorm stores its output in bf16 and writes that
BatchNorm's batch statistics in its epilogue; the dgrad producing a
BatchNorm's dY writes the BatchNorm's backward sums (ops/functional.py).
BatchNorm math, the native fp32 linear layers (gops::linear_fwd /
linear_bwd), gradients and the optimizer stay fp32.

On GPU one training step is: batch gather from the device-resident shard at
the device step offset -> forward/backward through the native NHWC kernels
(parameter grads land directly in the flat grad buffer; with world > 1 each
gradient bucket is all-reduced over RCCL on a comm stream as soon as backward
has completed it, parallel/overlap.py) -> device LR -> flat SGD kernel (which
bumps the device step).
Nothing in the step touches the host, so G steps are captured into one
hipGraph (torch.cuda.CUDAGraph) after a short eager warm-up and replayed.
On CPU the same model runs through the PyTorch oracle ops.
"""

from __future__ import annotations

import dataclasses
import gc

from typing import Optional

import numpy as np
import torch

from .. import config as C
from ..models.generic import make_model
from ..ops import functional as Fn
from ..ops import native, ptr, stream_handle
from ..parallel.comm import DeviceComm, all_reduce_grads_
from ..parallel.overlap import BUCKET_PLANS, BucketedAllReduce, SegmentedStep, plan_layout
from ..utils.data import batch_offset
from ..utils.devcache import DeviceArrayCache
from ..utils.schedule import learning_rate


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


TUNE_REPLAYS = 2  # timed graph replays per bucket-plan candidate (after one untimed)


class GenericEngine:
    kind = "generic"

    def __init__(self, cfg: C.TrainConfig, train_x: np.ndarray, train_y: np.ndarray,
                 device: torch.device, rank: int = 0, world: int = 1,
                 comm: Optional[DeviceComm] = None, force_sync: bool = False,
                 oracle: bool = False):
        """oracle: run the model through the PyTorch ops (F.conv2d,
        F.batch_norm, autograd) on `device` - a GPU-resident fp32 reference
        run of the same init, data and batch order (ops/functional.py
        oracle_mode); always fp32, eager, unsynced."""
        self.cfg, self.device, self.rank, self.world, self.comm = cfg, device, rank, world, comm
        self.oracle = bool(oracle)
        self.bf16 = cfg.dtype == "bf16"
        if self.oracle and (self.bf16 or world > 1):
            raise ValueError("the oracle engine is fp32 and single-rank")
        if self.bf16 and device.type != "cuda":
            raise NotImplementedError("dtype bf16 needs the GPU kernels (bf16 MFMA convolutions)")
        self.model = make_model(cfg.model)
        self.layout = self.model.layout
        self.B = cfg.batch_size
        self.n_local = int(train_x.shape[0])
        if self.n_local <= self.B:
            raise ValueError("local shard must exceed the batch")
        host = torch.zeros(self.layout.total)
        self.model.init_params(host, cfg.seed)
        self.params = host.to(device).requires_grad_(True)
        # zero state built on the host and copied: no device fill kernels (the
        # profiles' only at::native launches were these start-up fills)
        self.grads = torch.zeros(self.layout.total).to(device)
        self.mom = torch.zeros(self.layout.total).to(device)
        pv = self.layout.views(self.params)
        gv = self.layout.views(self.grads)
        self.P = {s.name: Fn.Param(pv[s.name], gv[s.name]) for s in self.layout.specs}
        self.bn = self.model.make_bn_state(device)
        self.train_x = torch.from_numpy(np.ascontiguousarray(train_x, np.float32)).to(device)
        self.train_y = torch.from_numpy(np.asarray(train_y).astype(np.int32)).to(device)
        self.step = 0
        self.grad_sync = cfg.sync == "grad" and world > 1 and comm is not None
        if force_sync and comm is not None:  # exercise the collective path at world 1
            self.grad_sync = True
        self.on_gpu = device.type == "cuda" and not self.oracle
        self.wcache = None
        self.use_graph = cfg.graph and self.on_gpu
        self.graph_steps = max(1, cfg.graph_steps)
        self._graphs = {}
        self._graph_loss = {}
        self._warm = False
        self.loss_buf = torch.zeros(()).to(device)
        self._eval_x = DeviceArrayCache()
        self.bucketer = None
        self.bucket_plan = None
        self._tuned = cfg.bucket_plan != "auto"
        self.tune_log = {}
        self.tune_steps_run = 0
        if self.on_gpu:
            self._C = native()
            if self.grad_sync:
                if comm.native_handle is None:
                    raise RuntimeError("GPU grad sync needs the native RCCL communicator")
                self.bucket_plan = "layout" if cfg.bucket_plan == "auto" else cfg.bucket_plan
                self.bucketer = self._make_bucketer(self.bucket_plan)
                comm.all_reduce_(self.grads)  # connection setup outside any capture
                torch.cuda.synchronize(device)
            h, w, c = train_x.shape[1:]
            self.xb = torch.empty(self.B, h, w, c, device=device)
            self.yb = torch.empty(self.B, dtype=torch.int32, device=device)
            self.step_dev = torch.zeros(1, dtype=torch.int64).to(device)
            self.lr_dev = torch.zeros(1).to(device)
            self.seed = torch.ones(()).to(device)  # backward seed, never written
            # the conv weights' re-laid copies (bf16 MFMA layouts; fp32: the
            # flipped stride-1 dgrad weights), written by the step's SGD launch
            # (ConvWeightCopies.sgd) and re-derived at the start of a run
            self.wcache = Fn.ConvWeightCopies(self.P, device, flat=self.params,
                                              kind="bf16" if self.bf16 else "f32flip")
            if self.wcache.njobs == 0:  # (LeNet-5 etc.: nothing to keep)
                self.wcache = None
            self._wfresh = False  # the copies match the fp32 weights

    # ------------------------------------------------------------------ util
    @property
    def sync_schedule(self) -> str:
        return f"buckets({self.bucket_plan})" if self.bucketer is not None else "n/a"

    def _make_bucketer(self, plan: str) -> BucketedAllReduce:
        # every plan runs on the same comm stream (a new stream could land on
        # another hardware queue and time differently for that alone)
        stream = self.bucketer.stream if self.bucketer is not None else None
        return BucketedAllReduce(plan_layout(self.layout, plan), self.grads, self.comm,
                                 self.device, wire=self.cfg.grad_comm_dtype, stream=stream)

    def _set_bucket_plan(self, plan: str) -> None:
        """Switches the all-reduce bucketing; the captured graphs (which hold
        the old buckets' events and collectives) are dropped."""
        if plan == self.bucket_plan:
            return
        torch.cuda.synchronize(self.device)
        self.bucketer = self._make_bucketer(plan)
        self.bucket_plan = plan
        self._graphs.clear()
        self._graph_loss.clear()
        gc.collect()  # the dropped graphs go now, never inside a later capture

    def tune_schedule(self) -> int:
        """cfg.bucket_plan == "auto" with a bucketed all-reduce: times
        TUNE_REPLAYS graph replays of every overlap/BUCKET_PLANS candidate
        (after one untimed replay each) on the real communicator and keeps the
        fastest - how much of the gradient all-reduce hides under backward
        depends on the link speed, the rank count and what a live second
        stream costs the graph, so the bucket count is measured, not fixed
        (PERF_NOTES "ResNet-18 all-reduce buckets").  Collective over the
        ranks: every rank times the same candidates in the same order and
        decides from the max-over-ranks times.  Side-effect free: params,
        momentum, BatchNorm running statistics and the step are restored, so
        the trial steps do not count.  Returns the number of trial steps."""
        if self._tuned or self.bucketer is None or not self.use_graph:
            self._tuned = True
            return 0
        from ..parallel import dist as D
        G = self.graph_steps
        host_step = self.step
        snap = (self.params.detach().clone(), self.mom.clone(), self.step_dev.clone(),
                {k: (rm.clone(), rv.clone()) for k, (rm, rv) in self.bn.items()})
        self._warmup(3)  # the capture precondition; its steps are undone below too
        seen, best, steps = {}, None, 0
        for plan in BUCKET_PLANS:
            key = tuple(plan_layout(self.layout, plan).buckets())
            if key in seen:  # same cut as an earlier candidate
                self.tune_log[plan] = self.tune_log[seen[key]]
                continue
            seen[key] = plan
            self._set_bucket_plan(plan)
            g = self._graph(G)
            if D.allreduce_max_host(0.0 if g is not None else 1.0) != 0.0:
                self.use_graph = False  # some rank could not capture: every rank runs eagerly
                best = None
                break
            g.replay()
            t0 = torch.cuda.Event(enable_timing=True)
            t1 = torch.cuda.Event(enable_timing=True)
            t0.record()
            for _ in range(TUNE_REPLAYS):
                g.replay()
            t1.record()
            torch.cuda.synchronize(self.device)
            steps += (1 + TUNE_REPLAYS) * G
            us = D.allreduce_max_host(1000.0 * t0.elapsed_time(t1) / (TUNE_REPLAYS * G))
            self.tune_log[plan] = round(us, 1)
            if best is None or us < best[0]:
                best = (us, plan)
        self._set_bucket_plan(best[1] if best is not None else "layout")
        self.params.data.copy_(snap[0])
        self.mom.copy_(snap[1])
        self.step_dev.copy_(snap[2])
        for k, (rm, rv) in snap[3].items():
            self.bn[k][0].copy_(rm)
            self.bn[k][1].copy_(rv)
        if self.wcache is not None:  # the bf16 weight copies follow the restored weights
            self.wcache.refresh()
            self._wfresh = True
        torch.cuda.synchronize(self.device)
        self.step = host_step
        self._tuned = True
        self.tune_steps_run = steps
        return steps

    def lr(self, step: Optional[int] = None) -> float:
        s = self.step if step is None else step
        return learning_rate(s, self.n_local, self.B, self.cfg.base_lr, self.cfg.lr_decay)

    def sync_optimizer_state(self) -> None:
        """Replicated optimizer state: nothing to gather."""

    def extra_state(self):
        """Non-trained model state saved with checkpoints: the BatchNorm
        running statistics under TF's names."""
        out = {}
        for name, (rm, rv) in self.bn.items():
            out[name + "/moving_mean"] = rm
            out[name + "/moving_variance"] = rv
        return out

    def set_step(self, step: int) -> None:
        self.step = int(step)
        if self.on_gpu:
            self.step_dev.copy_(torch.tensor([int(step)], dtype=torch.int64))

    def loss_value(self) -> float:
        t = getattr(self, "_loss_t", None) if self.on_gpu else None
        return float((t if t is not None else self.loss_buf).item())

    def param_views(self):
        return self.layout.views(self.params.detach())

    # ------------------------------------------------------------------ step
    def _step_gpu(self):
        if self.wcache is not None and not self._wfresh:
            self.wcache.refresh()
            self._wfresh = True
        gscale = self._forward_backward()
        self.update_gpu(gscale)

    def forward_backward_gpu(self) -> float:
        """Batch gather + forward + backward into the flat grad buffer (plus
        the bucketed all-reduce when syncing); returns the gradient scale the
        update must apply (1/world when the grads hold a cross-rank sum).
        Public entry (tests, serial emulations): the caller may have changed
        the weights, so the conv weight copies are re-derived first."""
        if self.wcache is not None:
            self.wcache.refresh()
            self._wfresh = True
        return self._forward_backward()

    def _forward_backward(self) -> float:
        C_ = self._C
        Fn.set_conv_bf16(self.bf16)
        s = stream_handle()
        row = int(np.prod(self.xb.shape[1:]))
        # the gather also writes this step's device LR (no separate LR launch)
        C_.ops.gather_batch(ptr(self.train_x), ptr(self.train_y), ptr(self.step_dev), self.n_local,
                            self.B, row, ptr(self.xb), ptr(self.yb), s, self.cfg.base_lr,
                            self.cfg.lr_decay, ptr(self.lr_dev))
        self._lr_fresh = True
        logits = self.model.forward(self.P, self.bn, self.xb, True)
        loss = Fn.cross_entropy(logits, self.yb)
        # keep the device scalar itself (no copy launch): under graph capture its
        # storage is the graph's, rewritten by every replay
        self._loss_t = loss.detach()
        gscale = 1.0
        Fn.set_unit_loss_seed(True)
        try:
            if self.bucketer is not None:
                # buckets all-reduce on the comm stream as backward completes them
                self.bucketer.begin()
                Fn.set_grad_hook(self.bucketer.grad_ready)
                try:
                    loss.backward(self.seed)
                finally:
                    Fn.set_grad_hook(None)
                self.bucketer.finish()
                gscale = 1.0 / self.world
            else:
                loss.backward(self.seed)
        finally:
            Fn.set_unit_loss_seed(False)
        return gscale

    def update_gpu(self, gscale: float) -> None:
        """The flat momentum SGD (which bumps the device step) at the device LR
        the step's batch gather wrote (or a separate LR launch when no gather
        of this step ran since the last update)."""
        C_ = self._C
        s = stream_handle()
        if not getattr(self, "_lr_fresh", False):
            C_.ops.lr_from_step(ptr(self.step_dev), self.n_local, self.B, self.cfg.base_lr,
                                self.cfg.lr_decay, ptr(self.lr_dev), s)
        self._lr_fresh = False
        if self.wcache is not None:  # + the bf16 layouts of the updated conv weights
            self.wcache.sgd(self.grads, self.mom, self.cfg.momentum, gscale, self.lr_dev,
                            self.step_dev)
            return
        C_.optim.sgd_momentum(ptr(self.params), ptr(self.grads), ptr(self.mom), self.layout.total, 0,
                              0.0, self.cfg.momentum, gscale, ptr(self.lr_dev), 0.0,
                              ptr(self.step_dev), s)

    def _step_cpu(self):
        off = batch_offset(self.step, self.n_local, self.B)
        x = self.train_x[off:off + self.B]
        y = self.train_y[off:off + self.B]
        self.params.grad = None
        logits = self.model.forward(self.P, self.bn, x, True)
        loss = Fn.cross_entropy(logits, y)
        loss.backward()
        with torch.no_grad():
            self.grads.copy_(self.params.grad)
            self.loss_buf.copy_(loss.detach())
            if self.grad_sync:
                all_reduce_grads_(self.comm, self.grads, self.cfg.grad_comm_dtype)
                self.grads.mul_(1.0 / self.world)
            self.mom.mul_(self.cfg.momentum).add_(self.grads)
            self.params.sub_(self.lr() * self.mom)

    def _segmented(self) -> bool:
        return self.bucketer is not None and len(self.bucketer.slices) > 1

    def _seg_graph(self, n: int):
        """n steps as linear compute segments + per-bucket collective graphs
        (parallel/overlap.py SegmentedStep): one step's optimizer and the
        next step's forward share a segment, so a step pays one graph
        boundary per overlapped bucket and nothing between steps."""
        g = self._graphs.get(n)
        if g is not None:
            return g
        # (as torch.cuda.graph does: collect before capturing - a graph or an
        # event freed by a collection inside the capture aborts the process -
        # and keep the collector off until the capture has ended)
        gc.collect()
        torch.cuda.synchronize(self.device)
        cap = torch.cuda.Stream(device=self.device)
        cap.wait_stream(torch.cuda.current_stream())
        host = self._host_state()
        seg = SegmentedStep(self.bucketer.stream, torch.cuda.graph_pool_handle(),
                            lambda st: self._C.capture_node_count(stream_handle(st)))
        self.bucketer.segment = seg
        err = None
        gc_was_on = gc.isenabled()
        gc.disable()
        with torch.cuda.stream(cap):
            try:
                seg.begin()
                for _ in range(n):
                    self._step_gpu()
                seg.end()
            except RuntimeError as e:
                err = e
                if seg.cur is not None:  # leave no capture open on the stream
                    try:
                        seg.cur.capture_end()
                    except RuntimeError:
                        pass
            finally:
                self.bucketer.segment = None
                if gc_was_on:
                    gc.enable()
        torch.cuda.current_stream().wait_stream(cap)
        if not self._capture_voted(err, host, "segmented hipGraph capture"):
            return None
        self._graphs[n] = seg
        self._graph_loss[n] = self._loss_t
        return seg

    def _graph(self, n: int):
        if self._segmented():
            return self._seg_graph(n)
        g = self._graphs.get(n)
        if g is None:
            g = torch.cuda.CUDAGraph()
            host = self._host_state()
            err = None
            try:
                with torch.cuda.graph(g):
                    for _ in range(n):
                        self._step_gpu()
            except RuntimeError as e:
                err = e
            if not self._capture_voted(err, host, "hipGraph capture"):
                return None
            self._graphs[n] = g
            # the loss tensor of the LAST step in this graph: its storage
            # belongs to the graph and is rewritten by every replay
            self._graph_loss[n] = self._loss_t
        return g

    def collective_graph_nodes(self):
        """Per overlapped (non-final) bucket of the longest captured segmented
        graph: the nodes its collective graph captured (None without one)."""
        segs = [v for k, v in sorted(self._graphs.items()) if isinstance(v, SegmentedStep)]
        return segs[-1].collective_nodes() if segs else None

    def _host_state(self):
        """Host-side state a captured step changes (the bucketer resets its own
        per-step state in begin()): restored when a capture is abandoned."""
        return (getattr(self, "_loss_t", None), self._wfresh, getattr(self, "_lr_fresh", False))

    def _capture_voted(self, err, host, what: str) -> bool:
        """Collective: a capture is kept only if it succeeded on EVERY rank
        (a rank training eagerly next to captured peers would issue its
        collectives on another schedule); otherwise every rank restores the
        host state the aborted capture changed and trains eagerly."""
        ok = err is None
        if self.world > 1 and self.comm is not None:
            from ..parallel import dist as D
            ok = D.allreduce_max_host(0.0 if ok else 1.0) == 0.0
        if ok:
            return True
        why = err if err is not None else "it failed on another rank"
        print(f"[rank {self.rank}] {what} failed ({why}); using eager launches", flush=True)
        self._loss_t, self._wfresh, self._lr_fresh = host
        self.use_graph = False
        torch.cuda.synchronize(self.device)
        return False

    def _warmup(self, k: int) -> int:
        """Eager warm-up on a side stream before the first capture (torch's
        documented requirement for capturing autograd); real training steps.
        Returns how many it ran."""
        if not self.use_graph or self._warm or k <= 0:
            return 0
        n = min(3, k)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(n):
                self._step_gpu()
        torch.cuda.current_stream().wait_stream(s)
        self._warm = True
        self.step += n
        return n

    def capture(self, k: int) -> None:
        """Pre-captures the graphs `train(k)` will replay (G-step graph and the
        k % G remainder), so a timed train(k) launches only graph replays.  May
        run the (untimed) eager warm-up steps first."""
        if not (self.on_gpu and self.use_graph) or k <= 0:
            return
        self._warmup(3)
        G = self.graph_steps
        if k >= G:
            self._graph(G)
        if k % G:
            self._graph(k % G)

    def train(self, k: int) -> None:
        if k <= 0:
            return
        if not self.on_gpu:
            with Fn.oracle_mode() if self.oracle else _null():
                for _ in range(k):
                    self._step_cpu()
                    self.step += 1
            return
        if self.wcache is not None:
            # the weights may have changed since the last step (init, checkpoint,
            # parameter averaging): re-derive the bf16 layouts once; the steps'
            # SGD launches keep them current from here on
            self.wcache.refresh()
            self._wfresh = True
        left = k - self._warmup(k)
        if not self.use_graph:
            for _ in range(left):
                self._step_gpu()
        else:
            G = self.graph_steps
            full, rem = divmod(left, G)
            g = self._graph(G) if full else None
            if g is not None:
                for _ in range(full):
                    g.replay()
                self._loss_t = self._graph_loss[G]
            else:
                rem = left
            gr = self._graphs.get(rem) if (rem and self.use_graph) else None
            if gr is not None:  # remainder graph pre-captured by capture()
                gr.replay()
                self._loss_t = self._graph_loss[rem]
            else:
                for _ in range(rem):  # remainder eagerly (avoids capturing odd sizes)
                    self._step_gpu()
        self.step += left

    # ------------------------------------------------------------------ eval
    @torch.no_grad()
    def evaluate(self, x: np.ndarray, y: np.ndarray, chunk: int = 256, dropout: bool = False,
                 return_logits: bool = False):
        n = int(x.shape[0])
        outs = []
        if not self.on_gpu:
            wrong = 0
            with Fn.oracle_mode() if self.oracle else _null():
                for a in range(0, n, chunk):
                    xb = torch.from_numpy(np.ascontiguousarray(x[a:a + chunk], np.float32))
                    lg = self.model.forward(self.P, self.bn, xb.to(self.device), False)
                    if return_logits:
                        outs.append(lg)
                    pred = lg.argmax(1).cpu().numpy()
                    wrong += int((pred != y[a:a + chunk]).sum())
            err = 100.0 * wrong / max(1, n)
            return (err, torch.cat(outs)) if return_logits else err
        # GPU: the test set is uploaded once and stays resident; the xent
        # kernel's argmax counter accumulates the correct predictions on the
        # device, so the whole evaluation ends in ONE 4-byte read
        Fn.set_conv_bf16(self.bf16)
        xd = self._eval_x.get(x, self.device)
        yd = torch.from_numpy(np.asarray(y).astype(np.int32)).to(self.device)
        correct = torch.zeros(1, dtype=torch.int32, device=self.device)
        s = stream_handle()
        if self.wcache is not None:
            self.wcache.refresh()
        for a in range(0, n, chunk):
            xb, yb = xd[a:a + chunk], yd[a:a + chunk]
            logits = self.model.forward(self.P, self.bn, xb, False).contiguous()
            if return_logits:
                outs.append(logits)
            m, k = logits.shape
            rows = torch.empty(m, device=self.device)
            self._C.ops.xent(ptr(logits), ptr(yb), m, k, ptr(rows), 0, ptr(correct), s)
        err = 100.0 * (n - int(correct.item())) / max(1, n)
        return (err, torch.cat(outs)) if return_logits else err


def make_image_engine(cfg: C.TrainConfig, train_x: np.ndarray, train_y: np.ndarray,
                      device: torch.device, rank: int = 0, world: int = 1,
                      comm: Optional[DeviceComm] = None, force_sync: bool = False,
                      xcomm=None):
    """Engine for the extra image models: LeNet-5 on a GPU runs the fused
    two-launch executor (runtime/lenet_engine.py); everything else (ResNet-18,
    the CPU oracle) runs the op-by-op engine.  LeNet-5 has no bf16 variant:
    its 3- and 6-channel convs and its FCs are VALU work whatever the operand
    type (the op-by-op engine's "bf16" LeNet ran the same fp32 math 6x
    slower), so --dtype bf16 runs the fp32 executor, says so, and the
    engine's `dtype` reports fp32."""
    if cfg.model == "lenet5" and device.type == "cuda":
        from .lenet_engine import NativeLenetEngine

        if cfg.dtype != "fp32":
            if rank == 0:
                print("[lenet5] --dtype bf16: LeNet-5's layers are VALU-bound at any operand "
                      "type; running the fp32 fused executor", flush=True)
            cfg = dataclasses.replace(cfg, dtype="fp32")
        return NativeLenetEngine(cfg, train_x, train_y, device, rank, world, comm, force_sync,
                                 xcomm=xcomm)
    return GenericEngine(cfg, train_x, train_y, device, rank, world, comm, force_sync)
