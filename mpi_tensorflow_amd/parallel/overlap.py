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

All of it is stream/event work, so it is captured into the step's hipGraph
together with the compute (the RCCL communicator must have run once before
capture: connection setup is not capturable).
"""

from __future__ import annotations

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

    def begin(self) -> None:
        self.count = [0] * len(self.slices)
        self.launched = [False] * len(self.slices)
        self.order = []

    def _launch(self, b: int) -> None:
        self.launched[b] = True
        self.order.append(b)
        if len(self.slices) == 1:  # one bucket: no overlap to gain, no cross-queue hop
            all_reduce_grads_(self.comm, self.slices[b], self.wire,
                              stream=torch.cuda.current_stream(), stage=self.stage[b])
            return
        ev = self.events[b]
        ev.record(torch.cuda.current_stream())
        self.stream.wait_event(ev)
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
        if len(self.slices) > 1:
            torch.cuda.current_stream().wait_stream(self.stream)
