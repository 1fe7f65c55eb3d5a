"""The reference's 2-layer MNIST CNN: parameter schema, init, and the fp32
PyTorch oracle forward / loss.

Reference (`/root/reference/mpipy.py`):
  * parameters `:38-53` (HWIO conv weights, [in, out] FC weights,
    truncated_normal(stddev=0.1, seed=1) weights, zeros/0.1 biases)
  * forward `Cnn.model` `:155-167`: conv5x5(1->32, SAME) + bias, ReLU,
    maxpool 2x2/2 -> conv5x5(32->64) + bias, ReLU, maxpool -> reshape
    [B, 7*7*64] in (h, w, c) order -> FC 3136->512 + bias, ReLU -> dropout
    keep 0.5 -> FC 512->10 + bias
  * loss `:54-58`: mean sparse softmax cross-entropy + 5e-4 * (l2(fc1_w) +
    l2(fc1_b) + l2(fc2_w) + l2(fc2_b)), l2(x) = sum(x^2) / 2
  * heads `:67-68`: softmax(logits)

Activations are NHWC throughout, like the reference; the oracle permutes
to NCHW only to call `F.conv2d`.  The MI355X training step does NOT use
this module: it runs the fused HIP kernels of `ops/` through the executor
in `runtime/mnist_engine.py` (NativeMnistEngine, kernels in `csrc/kernels/mnist.hip`); this file is the numerics oracle and the
CPU/gloo (BASELINE config 1) path.
"""

from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.nn.functional as F

from .. import config as C
from ..parallel.flat import FlatLayout, ParamSpec

H1 = 32  # conv1 output channels
H2 = 64  # conv2 output channels
FC1_IN = (C.IMAGE_SIZE // 4) * (C.IMAGE_SIZE // 4) * H2  # 3136
FC1_OUT = 512

# creation order = TF auto-names
SPECS_CREATION = [
    ParamSpec("conv1_weight", "Variable", (5, 5, 1, H1), "trunc_normal", bucket=1),
    ParamSpec("conv1_bias", "Variable_1", (H1,), "zeros", bucket=1),
    ParamSpec("conv2_weight", "Variable_2", (5, 5, H1, H2), "trunc_normal", bucket=1),
    ParamSpec("conv2_bias", "Variable_3", (H2,), "const:0.1", bucket=1),
    ParamSpec("fc1_weight", "Variable_4", (FC1_IN, FC1_OUT), "trunc_normal", l2=True, bucket=0),
    ParamSpec("fc1_bias", "Variable_5", (FC1_OUT,), "const:0.1", l2=True, bucket=0),
    ParamSpec("fc2_weight", "Variable_6", (FC1_OUT, C.NUM_CLASSES), "trunc_normal", l2=True, bucket=0),
    ParamSpec("fc2_bias", "Variable_7", (C.NUM_CLASSES,), "const:0.1", l2=True, bucket=0),
]
# flat buffer order: reverse of forward = order backward finishes them
FLAT_ORDER = ["fc2_weight", "fc2_bias", "fc1_weight", "fc1_bias",
              "conv2_weight", "conv2_bias", "conv1_weight", "conv1_bias"]


def layout() -> FlatLayout:
    by_name = {s.name: s for s in SPECS_CREATION}
    return FlatLayout.build([by_name[n] for n in FLAT_ORDER])


def init_params(flat: torch.Tensor, lay: FlatLayout, seed: int = C.SEED,
                stddev: float = C.INIT_STDDEV) -> None:
    """Deterministic init of the flat param buffer (same on every rank, so
    replicas start in sync without a broadcast - the reference relies on
    identical op seeds for the same effect, mpipy.py:40-52).  TF's Philox
    truncated-normal stream itself cannot be bit-matched."""
    flat.zero_()
    views = lay.views(flat)
    g = torch.Generator(device="cpu").manual_seed(seed)
    for s in SPECS_CREATION:  # creation order so the stream is stable
        v = views[s.name]
        if s.init == "trunc_normal":
            t = torch.empty(s.shape, dtype=torch.float32)
            torch.nn.init.trunc_normal_(t, 0.0, stddev, -2 * stddev, 2 * stddev, generator=g)
            v.copy_(t)
        elif s.init == "zeros":
            v.zero_()
        elif s.init.startswith("const:"):
            v.fill_(float(s.init.split(":", 1)[1]))
        else:
            raise ValueError(s.init)


def _nchw_w(w_hwio: torch.Tensor) -> torch.Tensor:
    return w_hwio.permute(3, 2, 0, 1)


def forward_features(p: Dict[str, torch.Tensor], x: torch.Tensor) -> torch.Tensor:
    """x [B,28,28,1] NHWC -> flattened pool2 output [B, 3136] in (h,w,c) order."""
    xn = x.permute(0, 3, 1, 2)
    z1 = F.conv2d(xn, _nchw_w(p["conv1_weight"]), p["conv1_bias"], padding=2)
    a1 = F.max_pool2d(F.relu(z1), 2, 2)
    z2 = F.conv2d(a1, _nchw_w(p["conv2_weight"]), p["conv2_bias"], padding=2)
    a2 = F.max_pool2d(F.relu(z2), 2, 2)
    return a2.permute(0, 2, 3, 1).reshape(x.shape[0], FC1_IN)


def forward(p: Dict[str, torch.Tensor], x: torch.Tensor, keep_mask: Optional[torch.Tensor] = None,
            keep_prob: float = C.DROPOUT_KEEP) -> torch.Tensor:
    """Logits [B,10].  `keep_mask` ([B,512] bool) applies dropout as TF1
    does: kept units scaled by 1/keep_prob, dropped units zero."""
    flat = forward_features(p, x)
    h = F.relu(flat @ p["fc1_weight"] + p["fc1_bias"])
    if keep_mask is not None:
        h = h * keep_mask.to(h.dtype) * (1.0 / keep_prob)
    return h @ p["fc2_weight"] + p["fc2_bias"]


def l2_term(p: Dict[str, torch.Tensor]) -> torch.Tensor:
    return sum(0.5 * (p[n] ** 2).sum() for n in ("fc1_weight", "fc1_bias", "fc2_weight", "fc2_bias"))


def loss_fn(p: Dict[str, torch.Tensor], logits: torch.Tensor, labels: torch.Tensor,
            l2: float = C.L2_COEF) -> torch.Tensor:
    """mpipy.py:54-58."""
    return F.cross_entropy(logits, labels.long()) + l2 * l2_term(p)
