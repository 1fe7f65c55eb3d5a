"""Checkpoint save / resume in the TF1 variable layout.

The reference never saves anything (no tf.train.Saver); the
trained model vanishes when its session closes (`/root/reference/mpipy.py:72-74`).
This module adds save/resume keyed by the names TF1 would have given the
reference's unnamed variables:

    Variable   conv1_weight [5,5,1,32]  HWIO      Variable_4 fc1_weight [3136,512]
    Variable_1 conv1_bias   [32]                  Variable_5 fc1_bias   [512]
    Variable_2 conv2_weight [5,5,32,64] HWIO      Variable_6 fc2_weight [512,10]
    Variable_3 conv2_bias   [64]                  Variable_7 fc2_bias   [10]
    Variable_8 iter_ (float32 global step)        <name>/Momentum  optimizer slots

Non-trained model state (the BatchNorm running statistics of ResNet-18) is
stored as extra named arrays under TF's names (`<bn>/moving_mean`,
`<bn>/moving_variance`).  Because TF's float32 `iter_` rounds above 2^24,
the exact step is also kept as int64 under `__meta__/step` and read first.
On resume, a checkpoint written by a different model or world size is
rejected (the LR decay period and the shard sizes depend on the world size,
mpipy.py:62, :211) unless the caller explicitly allows it.

Files are `.npz` (numpy, no pickle - loadable with allow_pickle=False) written
by rank 0 via a temp file + atomic rename.
"""

from __future__ import annotations

import os
import warnings
from typing import Dict, Mapping, Optional, Tuple

import numpy as np
import torch

from ..parallel.flat import FlatLayout

STEP_NAME = "Variable_8"
META_PREFIX = "__meta__/"
STEP_META = META_PREFIX + "step"


def to_arrays(layout: FlatLayout, params: torch.Tensor, mom: torch.Tensor, step: int,
              meta: Dict[str, str] = None,
              extra: Optional[Mapping[str, torch.Tensor]] = None) -> Dict[str, np.ndarray]:
    pv = layout.views(params.detach().float().cpu())
    mv = layout.views(mom.detach().float().cpu())
    out: Dict[str, np.ndarray] = {}
    for s in layout.specs:
        out[s.tf_name] = pv[s.name].numpy().copy()
        out[s.tf_name + "/Momentum"] = mv[s.name].numpy().copy()
    for k, t in (extra or {}).items():
        out[k] = t.detach().float().cpu().numpy().copy()
    out[STEP_NAME] = np.array(float(step), dtype=np.float32)
    out[STEP_META] = np.array(int(step), dtype=np.int64)
    for k, v in (meta or {}).items():
        out[META_PREFIX + k] = np.array(str(v))
    return out


def save(path: str, layout: FlatLayout, params: torch.Tensor, mom: torch.Tensor, step: int,
         meta: Dict[str, str] = None,
         extra: Optional[Mapping[str, torch.Tensor]] = None) -> str:
    arrays = to_arrays(layout, params, mom, step, meta, extra)
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = path + ".tmp.npz"
    np.savez(tmp, **arrays)
    os.replace(tmp, path)
    return path


@torch.no_grad()
def load(path: str, layout: FlatLayout, params: torch.Tensor, mom: torch.Tensor,
         extra: Optional[Mapping[str, torch.Tensor]] = None,
         expect: Optional[Mapping[str, object]] = None,
         strict_meta: bool = True) -> Tuple[int, Dict[str, str]]:
    """Loads into the flat buffers (and the `extra` tensors) in place;
    returns (step, meta).  `params` may be an autograd leaf: the copies run
    under no_grad on its storage.  `expect` (e.g. {"model": ..., "world": ...})
    is compared with the saved meta: a mismatch raises when `strict_meta`,
    else warns."""
    with np.load(path, allow_pickle=False) as z:
        meta = {k[len(META_PREFIX):]: str(z[k]) for k in z.files
                if k.startswith(META_PREFIX) and k != STEP_META}
        for k, want in (expect or {}).items():
            have = meta.get(k)
            if have is not None and have != str(want):
                msg = f"{path}: saved {k}={have} but this run has {k}={want}"
                if strict_meta:
                    raise ValueError(msg + " (the LR schedule / shards would change)")
                warnings.warn(msg)
        pv = layout.views(params.detach())
        mv = layout.views(mom.detach())
        for s in layout.specs:
            w = z[s.tf_name]
            if tuple(w.shape) != tuple(s.shape):
                raise ValueError(f"{path}: {s.tf_name} ({s.name}) has shape {w.shape}, expected {s.shape}")
            pv[s.name].copy_(torch.from_numpy(np.ascontiguousarray(w, np.float32)))
            key = s.tf_name + "/Momentum"
            if key in z.files:
                mv[s.name].copy_(torch.from_numpy(np.ascontiguousarray(z[key], np.float32)))
            else:
                mv[s.name].zero_()
        for k, t in (extra or {}).items():
            if k not in z.files:
                raise ValueError(f"{path}: missing model state {k}")
            a = z[k]
            if tuple(a.shape) != tuple(t.shape):
                raise ValueError(f"{path}: {k} has shape {a.shape}, expected {tuple(t.shape)}")
            t.copy_(torch.from_numpy(np.ascontiguousarray(a, np.float32)))
        if STEP_META in z.files:
            step = int(z[STEP_META])
        else:
            step = int(float(z[STEP_NAME])) if STEP_NAME in z.files else 0
    return step, meta
