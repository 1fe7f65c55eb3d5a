"""Backward-overlapped, bucketed gradient all-reduce for the generic models.

The reference averages weights with a blocking host-staged Gather every 50
steps (/root/reference/mpipy.py:91, :95-153); the DP default here is a
per-step gradient all-reduce.  For ResNet-18 (11.2 M params,
44.7 MB of fp32 grads) that all-reduce is large enough to matter, so it runs
in buckets on a dedicated comm stream while the backward pass continues:

* the flat grad buffer is laid out in reverse forward order (parallel/flat.py),
  so each bucket is one contiguous slice and buckets become complete in
  backward order;
* every backward kernel writes its parameter gradient straight into the flat
  buffer and then reports it (`ops.functional` grad hook); when the last
  parameter of a bucket has been reported, an event is recorded on the
  compute stream, the comm stream waits for it, and the bucket's in-place
  all-reduce is issued there;
* `finish()` issues any bucket that was never completed (parameters without
  a gradient this step) and joins the comm stream back into the compute
  stream before the optimizer;
* a model whose gradients fit in one bucket (models/generic.py BUCKET_BYTES:
  LeNet-5) all-reduces on the compute stream itself, after backward: a
  cross-queue fork + join would cost more than the overlap saves.

All of it is stream/event work.  Under graph capture the step with more than
one bucket is captured as linear compute segments with the collectives as
graphs of their own between them (SegmentedStep); a one-bucket step is one
linear graph.  The RCCL communicator must have run once before capture
(connection setup is not capturable).
"""

from __future__ import annotations

import warnings
from typing import Dict, List, Optional

import torch

from .comm import DeviceComm, all_reduce_grads_
from .flat import FlatLayout, _round_up

GEO_MIN_BYTES = 1 << 20  # geometric plans: no bucket cut below this many bytes
# the startup auto-tune's candidates (GenericEngine.tune_schedule); plans that
# cut a model's buckets identically are timed once
BUCKET_PLANS = ("layout", "one", "bytes:16", "geo:4", "geo:8")


def check_plan(plan: str) -> None:
    kind, _, arg = plan.partition(":")
    ok = (plan in ("layout", "one") or
          (kind in ("bytes", "geo") and arg.replace(".", "", 1).isdigit()
           and float(arg) > (1.0 if kind == "geo" else 0.0)))
    if not ok:
        raise ValueError(f"unknown bucket plan {plan!r} (auto / layout / one / bytes:MiB / "
                         "geo:RATIO>1)")


def plan_layout(layout: FlatLayout, plan: str) -> FlatLayout:
    """`layout` with its all-reduce buckets re-cut at parameter boundaries:

    * ``layout``  - the model's own buckets (models/generic.py BUCKET_BYTES);
    * ``one``     - a single bucket, reduced on the compute stream after backward;
    * ``bytes:M`` - buckets of ~M MiB each;
    * ``geo:R``   - geometric buckets from the front of the flat (backward)
      order, each 1/R of the one before: a CNN's deep stages hold most of the
      parameters and finish their backward first, so the first bucket is big
      and reduces under the rest of the backward, and the bucket left for the
      end of backward is small (ResNet-18, R=4: 33.6 / 8.4 / 2.7 MB = layer4 /
      layer3 / the rest).

    The flat order is unchanged; only the bucket ids move."""
    sizes = [4 * _round_up(s.numel) for s in layout.specs]
    total = sum(sizes)
    if plan == "layout":
        return layout
    if plan == "one":
        return layout.with_buckets([0] * len(sizes))
    kind, _, arg = plan.partition(":")
    if kind == "bytes":
        target = max(1, int(float(arg) * (1 << 20)))
        nb = max(1, -(-total // target))
        cuts = [total * (k + 1) / nb for k in range(nb - 1)]
    elif kind == "geo":
        r = float(arg)
        if r <= 1.0:
            raise ValueError(f"geometric bucket ratio must be > 1: {plan!r}")
        cuts, rest = [], float(total)
        while rest / r >= GEO_MIN_BYTES:  # the next cut leaves rest/r behind it
            rest /= r
            cuts.append(total - rest)
    else:
        raise ValueError(f"unknown bucket plan {plan!r}")
    ids, acc, b = [], 0, 0
    for sz in sizes:
        while b < len(cuts) and acc >= cuts[b]:
            b += 1
        ids.append(b)
        acc += sz
    dense = {v: i for i, v in enumerate(sorted(set(ids)))}  # (a big tensor skips ids)
    return layout.with_buckets([dense[v] for v in ids])


USE_DEV_EVENTS = True  # (A/B switch of scripts/seg_host_lab.py: torch's default events)


class DevEvent:
    """A stream-ordering event between two streams of one device: no timing
    and a device-scope release (csrc/bindings.cpp event_create).  A default
    event's system-scope fence writes back and invalidates the caches under
    the work after it."""

    def __init__(self):
        from ..ops import native

        self._C = native()
        self.h = self._C.event_create() if USE_DEV_EVENTS else None
        self.ev = None if USE_DEV_EVENTS else torch.cuda.Event()

    def record(self, stream: torch.cuda.Stream) -> None:
        if self.ev is not None:
            self.ev.record(stream)
        else:
            self._C.event_record(self.h, int(stream.cuda_stream))

    def wait(self, stream: torch.cuda.Stream) -> None:
        """`stream` waits for the work before the last record()."""
        if self.ev is not None:
            stream.wait_event(self.ev)
        else:
            self._C.stream_wait_event(int(stream.cuda_stream), self.h)

    def __del__(self):
        try:
            if self.h is not None:
                self._C.event_destroy(self.h)
        except Exception:  # interpreter shutdown
            pass


class SegmentedStep:
    """One training step captured as LINEAR compute graphs, with each gradient
    bucket's collective captured as a graph of its own on the comm stream in
    between, replayed with plain stream events.

    Why: a captured graph with a live second branch (the comm stream) makes HIP
    spread the graph's compute chain over the hardware queues.  That puts
    cross-queue hops on the critical path and slows the small kernels.
    ResNet-18 bf16 paid ~160 us a step for it with collectives that cost
    nothing (PERF_NOTES "ResNet-18 all-reduce buckets").  Linear segments keep
    the compute on one queue, and the collectives still overlap it.

    Capture protocol (GenericEngine._seg_graph): begin() on the capture stream;
    BucketedAllReduce calls cut() when a bucket is complete (from the backward
    ops' grad hook) and join() before the optimizer; end() after the step.
    `node_count(stream)` gives the nodes captured so far on a stream, so a
    segment is never closed empty: its cut's collective is chained after the
    previous one instead."""

    def __init__(self, comm_stream: torch.cuda.Stream, pool, node_count):
        self.comm_stream = comm_stream
        self.pool = pool
        self.node_count = node_count
        self.items: List[tuple] = []  # ("c", graph) | ("m", graph, event) | ("j",)
        self.cur: Optional[torch.cuda.CUDAGraph] = None

    def _open(self) -> None:
        # relaxed: a segment begun on one thread may end on the other (the
        # backward's grad hook runs on autograd's device thread)
        self.cur = torch.cuda.CUDAGraph()
        self.cur.capture_begin(pool=self.pool, capture_error_mode="relaxed")

    def _close(self, force: bool = False) -> bool:
        """Ends the open compute segment unless it is still empty (then it stays
        open, or with force is ended and dropped).  True if a segment was kept."""
        empty = self.node_count(torch.cuda.current_stream()) == 0
        if empty and not force:
            return False
        self.cur.capture_end()
        if not empty:
            self.items.append(("c", self.cur))
        self.cur = None
        return not empty

    def begin(self) -> None:
        self._open()

    def cut(self, collective) -> None:
        """Compute so far -> one segment; then `collective()` (launching on the
        comm stream) captured as its own graph."""
        closed = self._close()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(self.comm_stream):
            g.capture_begin(pool=self.pool, capture_error_mode="relaxed")
            collective()
            nodes = self.node_count(self.comm_stream)  # what this bucket's graph moves
            g.capture_end()
        self.items.append(("m", g, DevEvent(), nodes))
        if closed:
            self._open()

    def join(self) -> None:
        if self._close():
            self._open()
        self.items.append(("j", DevEvent()))

    def end(self) -> None:
        with warnings.catch_warnings():  # an empty last segment is ended and dropped
            warnings.filterwarnings("ignore", message="The CUDA Graph is empty")
            self._close(force=True)

    def collective_nodes(self) -> List[int]:
        """Nodes captured in each overlapped bucket's collective graph, in
        order (0 would be a collective that captured nothing: at world 1 the
        communicator returns at once; at N > 1 every one must move bytes)."""
        return [it[3] for it in self.items if it[0] == "m"]

    def replay(self) -> None:
        cs = torch.cuda.current_stream()
        for it in self.items:
            if it[0] == "c":
                it[1].replay()
            elif it[0] == "m":
                it[2].record(cs)
                it[2].wait(self.comm_stream)
                with torch.cuda.stream(self.comm_stream):
                    it[1].replay()
            else:
                it[1].record(self.comm_stream)
                it[1].wait(cs)


class BucketedAllReduce:
    def __init__(self, layout: FlatLayout, grads: torch.Tensor, comm: DeviceComm,
                 device: torch.device, wire: str = "fp32",
                 stream: Optional[torch.cuda.Stream] = None):
        self.comm = comm
        self.grads = grads
        self.wire = wire  # gradient wire dtype (TrainConfig.grad_comm_dtype)
        ranges = layout.buckets()  # [(lo, hi)] per bucket id, in flat order
        self.slices: List[torch.Tensor] = [grads[lo:hi] for lo, hi in ranges]
        self.stage: List[Optional[torch.Tensor]] = [None] * len(ranges)
        if wire == "bf16":  # bf16 staging per bucket (native conversions around the collective)
            st = torch.zeros(grads.numel(), dtype=torch.bfloat16, device=device)
            self.stage = [st[lo:hi] for lo, hi in ranges]
        views = layout.views(grads)
        self.bucket_of: Dict[int, int] = {}
        self.size = [0] * len(ranges)
        for s in layout.specs:
            self.bucket_of[views[s.name].data_ptr()] = s.bucket
            self.size[s.bucket] += 1
        self.stream = stream if stream is not None else torch.cuda.Stream(device=device)
        self.events = [torch.cuda.Event() for _ in ranges]
        self.count = [0] * len(ranges)
        self.launched = [False] * len(ranges)
        self.order: List[int] = []
        self.segment: Optional[SegmentedStep] = None  # set while a segmented step is captured
        self.dev_events: Optional[List[DevEvent]] = None  # eager steps' events (made on first use)
        self.joined = False
        self.eager_events = True

    def begin(self) -> None:
        self.count = [0] * len(self.slices)
        self.launched = [False] * len(self.slices)
        self.order = []
        self.joined = False
        # eager steps order the streams with device-scope events; a graph
        # capture turns torch's events into edges
        self.eager_events = not torch.cuda.is_current_stream_capturing()
        if self.eager_events and self.dev_events is None:
            self.dev_events = [DevEvent() for _ in self.slices]
            self.join_event = DevEvent()

    def _join(self) -> None:
        """The compute stream waits for the collectives issued so far."""
        self.joined = True
        if self.segment is not None:
            self.segment.join()
        elif self.eager_events:
            self.join_event.record(self.stream)
            self.join_event.wait(torch.cuda.current_stream())
        else:
            torch.cuda.current_stream().wait_stream(self.stream)

    def _launch(self, b: int) -> None:
        self.launched[b] = True
        self.order.append(b)
        # one bucket: no overlap to gain, no cross-queue hop.  The last bucket
        # of several: nothing is left to overlap it with, so join first and
        # reduce it on the compute stream (one hop back instead of a hop
        # there and one back after it)
        if len(self.slices) == 1 or len(self.order) == len(self.slices):
            if len(self.slices) > 1:
                self._join()
            all_reduce_grads_(self.comm, self.slices[b], self.wire,
                              stream=torch.cuda.current_stream(), stage=self.stage[b])
            return
        if self.segment is not None:
            self.segment.cut(lambda: all_reduce_grads_(self.comm, self.slices[b], self.wire,
                                                       stream=self.stream, stage=self.stage[b]))
            return
        if self.eager_events:
            self.dev_events[b].record(torch.cuda.current_stream())
            self.dev_events[b].wait(self.stream)
        else:  # under capture: torch's events become graph edges
            self.events[b].record(torch.cuda.current_stream())
            self.stream.wait_event(self.events[b])
        with torch.cuda.stream(self.stream):
            all_reduce_grads_(self.comm, self.slices[b], self.wire, stream=self.stream,
                              stage=self.stage[b])

    def grad_ready(self, grad_view: Optional[torch.Tensor]) -> None:
        if grad_view is None:
            return
        b = self.bucket_of.get(grad_view.data_ptr())
        if b is None:
            return
        self.count[b] += 1
        if self.count[b] == self.size[b] and not self.launched[b]:
            self._launch(b)

    def finish(self) -> None:
        for b in range(len(self.slices)):
            if not self.launched[b]:
                self._launch(b)
        if len(self.slices) > 1 and not self.joined:
            self._join()
