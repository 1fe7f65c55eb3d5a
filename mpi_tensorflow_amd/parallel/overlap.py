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
* the streams hand off through DEVICE FLAGS (csrc/kernels/streamflag.hip),
  not events: in graph replay an event fork / join whose branches run at once
  costs 15-18 us (scripts/microbench/edge_lab.hip, profiles/r5_edge_lab.txt),
  and the bucketed step had one per bucket.  The comm stream is forked from
  the compute stream once (first bucket of a run of steps) and joined once
  (`join()`, at the end of a captured graph / eager run); per bucket the
  compute stream signals a counter the comm stream's wait kernel polls, and
  `finish()` makes the compute stream wait on the comm stream's last signal.

All of it is stream/event work, so it is captured into the step's hipGraph
together with the compute (the RCCL communicator must have run once before
capture: connection setup is not capturable).
"""

from __future__ import annotations

from typing import Dict, List, Optional

import torch

from ..ops import native, ptr, stream_handle
from .comm import DeviceComm, all_reduce_grads_
from .flat import FlatLayout

FLAG_TIMEOUT_S = 30.0


class BucketedAllReduce:
    def __init__(self, layout: FlatLayout, grads: torch.Tensor, comm: DeviceComm,
                 device: torch.device, wire: str = "fp32", flags: bool = True):
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
        nb = len(ranges)
        self.use_flags = bool(flags) and nb > 1 and device.type == "cuda"
        # [0, nb]: signal counters (bucket b ready; nb: all buckets reduced),
        # [nb + 1, 2 nb + 1]: the waiters' expected counts, [2 nb + 2]: error bit
        self.fw = (torch.zeros(2 * nb + 3, dtype=torch.int32, device=device)
                   if self.use_flags else None)
        self._forked_from = None

    def _w(self, i: int) -> int:
        return ptr(self.fw) + 4 * i

    def error(self) -> int:
        """Sticky: 1 if a flag wait ever timed out (syncs the device)."""
        return int(self.fw[-1].item()) if self.fw is not None else 0

    def begin(self) -> None:
        self.count = [0] * len(self.slices)
        self.launched = [False] * len(self.slices)
        self.order = []
        if self.use_flags:  # fork the comm stream once per run of steps
            cur = torch.cuda.current_stream()
            if self._forked_from != cur:
                self.stream.wait_stream(cur)
                self._forked_from = cur

    def join(self) -> None:
        """Rejoins the comm stream into the current stream (end of a captured
        graph or of an eager run of steps; the flag waits ordered every step)."""
        if self.use_flags and self._forked_from is not None:
            torch.cuda.current_stream().wait_stream(self.stream)
            self._forked_from = None

    def _launch(self, b: int) -> None:
        self.launched[b] = True
        self.order.append(b)
        if len(self.slices) == 1:  # one bucket: no overlap to gain, no cross-queue hop
            all_reduce_grads_(self.comm, self.slices[b], self.wire,
                              stream=torch.cuda.current_stream(), stage=self.stage[b])
            return
        if self.use_flags:
            C = native()
            nb = len(self.slices)
            C.optim.flag_signal(self._w(b), stream_handle(torch.cuda.current_stream()))
            with torch.cuda.stream(self.stream):
                C.optim.flag_wait(self._w(b), self._w(nb + 1 + b), self._w(2 * nb + 2),
                                  FLAG_TIMEOUT_S, stream_handle(self.stream))
                all_reduce_grads_(self.comm, self.slices[b], self.wire, stream=self.stream,
                                  stage=self.stage[b])
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
            if self.use_flags:
                C = native()
                nb = len(self.slices)
                C.optim.flag_signal(self._w(nb), stream_handle(self.stream))
                C.optim.flag_wait(self._w(nb), self._w(2 * nb + 1), self._w(2 * nb + 2),
                                  FLAG_TIMEOUT_S, stream_handle(torch.cuda.current_stream()))
            else:
                torch.cuda.current_stream().wait_stream(self.stream)
