"""LeNet-5 (32x32x3) and ResNet-18 (224x224x3) on the generic NHWC op set -
the extra configs of BASELINE.json (configs 4 and 5: "LeNet-5 on synthetic
32x32x3 (CIFAR-shape)", "ResNet-18 on synthetic 224x224x3 ... stress MFMA
conv + all-reduce overlap").  The reference itself only trains the MNIST CNN
(/root/reference/mpipy.py:155-167); these models reuse its trainer contract
(flat buffers, reference LR schedule + momentum SGD, DP sync modes).

Each model is a parameter-spec list (laid out by parallel/flat.py in reverse
forward order, so all-reduce buckets follow backward completion) plus a
forward function over `Param` views; BatchNorm running statistics live in a
separate non-trained buffer.
"""

from __future__ import annotations

from typing import Dict, List, Tuple

import math
import torch

from ..ops import functional as Fn
from ..parallel.flat import FlatLayout, ParamSpec


def model_input_shape(name: str) -> Tuple[int, int, int]:
    return {"lenet5": (32, 32, 3), "resnet18": (224, 224, 3)}[name]


BUCKET_BYTES = 8 << 20  # target gradient bytes per all-reduce bucket
MAX_BUCKETS = 8


class GenericModel:
    name = "generic"
    num_classes = 10

    def __init__(self):
        self.specs: List[ParamSpec] = self._specs()
        # all-reduce buckets: contiguous groups in backward order (reverse
        # forward) of ~BUCKET_BYTES each.  Every extra bucket costs a
        # cross-queue fork/join (~5-10 us each in graph replay, PERF_NOTES),
        # so small models get ONE bucket, reduced on the compute stream.
        flat_order = list(reversed(self.specs))
        total = sum(4 * s.numel for s in flat_order)
        nb = max(1, min(MAX_BUCKETS, -(-total // BUCKET_BYTES)))
        sized, acc = [], 0
        ids: Dict[int, int] = {}  # dense bucket ids (a tensor larger than a bucket skips ids)
        for s in flat_order:
            b = min(nb - 1, (acc * nb) // total)
            acc += 4 * s.numel
            b = ids.setdefault(b, len(ids))
            sized.append(ParamSpec(s.name, s.tf_name, s.shape, s.init, s.l2, bucket=b))
        self.layout = FlatLayout.build(sized)
        self.bn_channels: Dict[str, int] = self._bn()

    # --- to override ---------------------------------------------------------
    def _specs(self) -> List[ParamSpec]:
        raise NotImplementedError

    def _bn(self) -> Dict[str, int]:
        return {}

    def forward(self, P: Dict[str, Fn.Param], bn: Dict[str, Tuple[torch.Tensor, torch.Tensor]],
                x: torch.Tensor, training: bool) -> torch.Tensor:
        raise NotImplementedError

    # --- shared --------------------------------------------------------------
    def init_params(self, flat: torch.Tensor, seed: int) -> None:
        flat.zero_()
        views = self.layout.views(flat)
        g = torch.Generator(device="cpu").manual_seed(seed)
        for s in self.specs:
            v = views[s.name]
            if s.init == "he_normal":
                fan_in = 1
                for d in s.shape[:-1]:
                    fan_in *= d
                t = torch.randn(s.shape, generator=g) * math.sqrt(2.0 / fan_in)
                v.copy_(t)
            elif s.init == "ones":
                v.fill_(1.0)
            elif s.init == "zeros":
                v.zero_()
            else:
                raise ValueError(s.init)

    def make_bn_state(self, device) -> Dict[str, Tuple[torch.Tensor, torch.Tensor]]:
        # built on the host and copied (no device fill kernels)
        return {k: (torch.zeros(c).to(device), torch.ones(c).to(device))
                for k, c in self.bn_channels.items()}


def _conv(name, r, cin, cout, bias=True):
    out = [ParamSpec(name + "_w", name + "/kernel", (r, r, cin, cout), "he_normal")]
    if bias:
        out.append(ParamSpec(name + "_b", name + "/bias", (cout,), "zeros"))
    return out


def _fc(name, fin, fout):
    return [ParamSpec(name + "_w", name + "/kernel", (fin, fout), "he_normal"),
            ParamSpec(name + "_b", name + "/bias", (fout,), "zeros")]


def _bnp(name, c):
    return [ParamSpec(name + "_g", name + "/gamma", (c,), "ones"),
            ParamSpec(name + "_b", name + "/beta", (c,), "zeros")]


class LeNet5(GenericModel):
    """conv5x5(3->6)+ReLU, maxpool2 -> conv5x5(6->16)+ReLU, maxpool2 ->
    FC 400->120+ReLU -> FC 120->84+ReLU -> FC 84->10 (valid convolutions)."""

    name = "lenet5"

    def _specs(self):
        return (_conv("c1", 5, 3, 6) + _conv("c2", 5, 6, 16) + _fc("f1", 400, 120) +
                _fc("f2", 120, 84) + _fc("f3", 84, 10))

    def forward(self, P, bn, x, training):
        h = Fn.conv2d(x, P["c1_w"], P["c1_b"], 1, 0, relu=True)
        h = Fn.maxpool(h, 2, 2)
        h = Fn.conv2d(h, P["c2_w"], P["c2_b"], 1, 0, relu=True)
        h = Fn.maxpool(h, 2, 2)
        h = h.reshape(h.shape[0], 400)
        h = Fn.linear(h, P["f1_w"], P["f1_b"], relu=True)
        h = Fn.linear(h, P["f2_w"], P["f2_b"], relu=True)
        return Fn.linear(h, P["f3_w"], P["f3_b"])


class ResNet18(GenericModel):
    """ResNet-18 (He et al. 2016), NHWC, BasicBlocks [2,2,2,2], 10 classes."""

    name = "resnet18"
    STAGES = [(64, 1), (128, 2), (256, 2), (512, 2)]

    def _blocks(self):
        cin = 64
        out = []
        for si, (c, stride) in enumerate(self.STAGES):
            for bi in range(2):
                s = stride if bi == 0 else 1
                out.append((f"l{si + 1}b{bi}", cin, c, s, s != 1 or cin != c))
                cin = c
        return out

    def _specs(self):
        sp = _conv("conv1", 7, 3, 64, bias=False) + _bnp("bn1", 64)
        for name, cin, c, s, down in self._blocks():
            sp += _conv(name + "c1", 3, cin, c, bias=False) + _bnp(name + "n1", c)
            sp += _conv(name + "c2", 3, c, c, bias=False) + _bnp(name + "n2", c)
            if down:
                sp += _conv(name + "ds", 1, cin, c, bias=False) + _bnp(name + "nd", c)
        sp += _fc("fc", 512, 10)
        return sp

    def _bn(self):
        d = {"bn1": 64}
        for name, cin, c, s, down in self._blocks():
            d[name + "n1"] = c
            d[name + "n2"] = c
            if down:
                d[name + "nd"] = c
        return d

    def forward(self, P, bn, x, training):
        # Every conv feeds a BatchNorm: in bf16 mode its output is stored bf16
        # (Fn.conv2d out_bf16; BN reads bf16 input), fp32 otherwise.  In training
        # each BatchNorm's statistics hand-offs are wired here, explicitly, by
        # one Fn.BnLink: the producing conv writes the forward sums (bn_out),
        # and the conv consuming the BatchNorm's output writes the backward sums
        # from its dgrad (bn_in) - n1 -> c2 inside a block, a block's n2 -> the
        # next block's c1 (whose dgrad also adds the shortcut's gradient, so its
        # dX is the BatchNorm's whole dY).
        links = {}

        def link(nm):
            if not (training and x.is_cuda):
                return None
            if nm not in links:
                links[nm] = Fn.BnLink(bn[nm][0] if Fn.BN_FWD_EPILOGUE else None)
            return links[nm]

        def out_link(nm):  # the producing conv's forward statistics
            lk = link(nm)
            return lk if (lk is not None and lk.shift is not None) else None

        def BN(h, nm, relu, res=None, res_join=None, twin_only=False):
            rm, rv = bn[nm]
            return Fn.batchnorm(h, P[nm + "_g"], P[nm + "_b"], rm, rv, training, relu, res,
                                res_join=res_join, twin_only=twin_only, link=link(nm))

        h = Fn.conv2d(x, P["conv1_w"], None, 2, 3, out_bf16=True, bn_out=out_link("bn1"))
        h = BN(h, "bn1", True, twin_only=True)  # the pool reads its bf16 twin
        h = Fn.maxpool(h, 3, 2, 1)
        join = x.is_cuda and training and torch.is_grad_enabled()
        h_bn = None  # the BatchNorm whose output h is (a block's n2)
        for name, cin, c, s, down in self._blocks():
            # the block input's two gradients (conv1, shortcut) meet in the
            # conv1 dgrad epilogue (Fn.GradJoin); the shortcut runs after c2
            # so its backward comes first
            j = Fn.GradJoin() if join else None
            o = Fn.conv2d(h, P[name + "c1_w"], None, s, 1, join=j, join_role="final",
                          out_bf16=True, bn_out=out_link(name + "n1"),
                          bn_in=link(h_bn) if h_bn else None)
            o = BN(o, name + "n1", True, twin_only=True)  # only conv c2 reads it
            o = Fn.conv2d(o, P[name + "c2_w"], None, 1, 1, out_bf16=True,
                          bn_out=out_link(name + "n2"), bn_in=link(name + "n1"))
            if down:
                sc = Fn.conv2d(h, P[name + "ds_w"], None, s, 0, join=j, join_role="stash",
                               out_bf16=True, bn_out=out_link(name + "nd"))
                h = BN(o, name + "n2", True, res=BN(sc, name + "nd", False))
            else:
                h = BN(o, name + "n2", True, res=h, res_join=j)
            h_bn = name + "n2"
        h = Fn.global_avgpool(h)
        return Fn.linear(h, P["fc_w"], P["fc_b"])


def make_model(name: str) -> GenericModel:
    return {"lenet5": LeNet5, "resnet18": ResNet18}[name]()
