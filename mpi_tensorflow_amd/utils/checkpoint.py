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

Files are `.npz` (numpy, no pickle - loadable with allow_pickle=False) written
by rank 0 via a temp file + atomic rename.
"""

from __future__ import annotations

import os
from typing import Dict, Tuple

import numpy as np
import torch

from ..parallel.flat import FlatLayout

STEP_NAME = "Variable_8"
META_PREFIX = "__meta__/"


def to_arrays(layout: FlatLayout, params: torch.Tensor, mom: torch.Tensor, step: int,
              meta: Dict[str, str] = None) -> Dict[str, np.ndarray]:
    pv = layout.views(params.detach().float().cpu())
    mv = layout.views(mom.detach().float().cpu())
    out: Dict[str, np.ndarray] = {}
    for s in layout.specs:
        out[s.tf_name] = pv[s.name].numpy().copy()
        out[s.tf_name + "/Momentum"] = mv[s.name].numpy().copy()
    out[STEP_NAME] = np.array(float(step), dtype=np.float32)
    for k, v in (meta or {}).items():
        out[META_PREFIX + k] = np.array(str(v))
    return out


def save(path: str, layout: FlatLayout, params: torch.Tensor, mom: torch.Tensor, step: int,
         meta: Dict[str, str] = None) -> str:
    arrays = to_arrays(layout, params, mom, step, meta)
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = path + ".tmp.npz"
    np.savez(tmp, **arrays)
    os.replace(tmp, path)
    return path


def load(path: str, layout: FlatLayout, params: torch.Tensor, mom: torch.Tensor) -> Tuple[int, Dict[str, str]]:
    """Loads into the flat buffers in place; returns (step, meta)."""
    with np.load(path, allow_pickle=False) as z:
        pv = layout.views(params)
        mv = layout.views(mom)
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
        step = int(float(z[STEP_NAME])) if STEP_NAME in z.files else 0
        meta = {k[len(META_PREFIX):]: str(z[k]) for k in z.files if k.startswith(META_PREFIX)}
    return step, meta
