"""Flat parameter / gradient / momentum buffers and all-reduce buckets.

The reference keeps nine separate TF variables (`/root/reference/mpipy.py:38-53`)
and moves four of them one by one through host numpy buffers for its
periodic Gather (`:121-127`).  Here all trainable tensors of a model live in
ONE contiguous fp32 buffer per role (param, grad, momentum):

* segments are laid out in REVERSE forward order, i.e. in the order the
  backward pass finishes them, so each all-reduce bucket is one contiguous
  slice that becomes ready as a unit (bucket 1 = FC params, ready after the
  fc1 backward kernel; bucket 2 = conv params, ready at the end);
* every segment starts on a 64-float (256 B) boundary so kernels can use
  16-byte vector access; the padding is zero in every role, so it is inert
  under all-reduce and SGD;
* per-tensor views keep the TF checkpoint layout (HWIO conv, [in, out] FC)
  and TF names (`Variable`, `Variable_1`, ... in creation order).
"""

from __future__ import annotations

import dataclasses
from typing import Dict, List, Sequence, Tuple

ALIGN = 64  # floats


def _round_up(x: int, a: int = ALIGN) -> int:
    return (x + a - 1) // a * a


@dataclasses.dataclass(frozen=True)
class ParamSpec:
    name: str  # attribute name in the reference (e.g. conv1_weight)
    tf_name: str  # TF1 auto-name in creation order (Variable, Variable_1, ...)
    shape: Tuple[int, ...]
    init: str  # "trunc_normal" | "zeros" | "const:<v>" | "ones" | "he_normal"
    l2: bool = False  # included in the L2 regulariser
    bucket: int = 0  # all-reduce bucket id (0 = first reduced)

    @property
    def numel(self) -> int:
        n = 1
        for s in self.shape:
            n *= s
        return n


@dataclasses.dataclass
class FlatLayout:
    specs: List[ParamSpec]  # in flat (reverse-forward) order
    offsets: Dict[str, int]
    total: int  # padded length in floats

    @classmethod
    def build(cls, specs_flat_order: Sequence[ParamSpec]) -> "FlatLayout":
        offs: Dict[str, int] = {}
        cur = 0
        for s in specs_flat_order:
            offs[s.name] = cur
            cur += _round_up(s.numel)
        return cls(list(specs_flat_order), offs, cur)

    @property
    def numel(self) -> int:
        """Real (unpadded) trainable parameter count."""
        return sum(s.numel for s in self.specs)

    def segment(self, name: str) -> Tuple[int, int]:
        s = self.spec(name)
        o = self.offsets[name]
        return o, o + s.numel

    def spec(self, name: str) -> ParamSpec:
        for s in self.specs:
            if s.name == name:
                return s
        raise KeyError(name)

    def views(self, flat) -> Dict[str, object]:
        """name -> view of `flat` (a 1-D torch tensor) with the param shape."""
        out = {}
        for s in self.specs:
            o = self.offsets[s.name]
            out[s.name] = flat[o:o + s.numel].view(s.shape)
        return out

    def buckets(self) -> List[Tuple[int, int]]:
        """Contiguous [start, stop) slices per bucket id, in reduce order."""
        res: Dict[int, List[int]] = {}
        for s in self.specs:
            o = self.offsets[s.name]
            lo_hi = res.setdefault(s.bucket, [o, o + _round_up(s.numel)])
            lo_hi[0] = min(lo_hi[0], o)
            lo_hi[1] = max(lo_hi[1], o + _round_up(s.numel))
        out = [tuple(res[k]) for k in sorted(res)]
        # buckets must tile the buffer contiguously
        cur = 0
        for lo, hi in out:
            if lo != cur:
                raise ValueError("bucket slices are not contiguous; check spec order")
            cur = hi
        if cur != self.total:
            raise ValueError("buckets do not cover the flat buffer")
        return out  # type: ignore[return-value]

    def with_buckets(self, ids: Sequence[int]) -> "FlatLayout":
        """The same segments with new bucket ids (one per spec, flat order)."""
        specs = [dataclasses.replace(s, bucket=int(b)) for s, b in zip(self.specs, ids, strict=True)]
        return FlatLayout(specs, dict(self.offsets), self.total)

    def l2_range(self) -> Tuple[int, int]:
        """[0, end) of the L2-regularised prefix (specs with l2=True must
        come first in flat order)."""
        end = 0
        seen_non_l2 = False
        for s in self.specs:
            if s.l2:
                if seen_non_l2:
                    raise ValueError("L2-regularised segments must be a prefix")
                end = self.offsets[s.name] + _round_up(s.numel)
            else:
                seen_non_l2 = True
        return 0, end

    def tf_names(self) -> Dict[str, str]:
        return {s.name: s.tf_name for s in self.specs}
