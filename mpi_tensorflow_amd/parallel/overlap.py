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
from .flat import FlatLayout


class BucketedAllReduce:
    def __init__(self, layout: FlatLayout, grads: torch.Tensor, comm: DeviceComm,
                 device: torch.device, wire: str = "fp32"):
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
        self.stream = torch.cuda.Stream(device=device)
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
