"""Autograd layer ops for the generic models (LeNet-5, ResNet-18).

Two implementations with identical math, chosen by the device of the input:

* GPU (`x.is_cuda`): the hand-written gfx950 kernels of
  `csrc/kernels/ops_generic.hip` through `_C.ops` - NHWC implicit-GEMM conv
  on fp32 MFMA (bias + ReLU fused), BatchNorm with the residual add + ReLU
  fused, max / average pooling, fused softmax cross-entropy.  Parameter
  gradients are written by the kernels STRAIGHT into the caller's flat grad
  buffer views (`Param.grad_view`), so a finished backward leaves the
  all-reduce buckets ready with no extra copies; the autograd functions
  return None for parameters.
* CPU: the plain-PyTorch fp32 oracle of the same ops (NCHW permutes around
  torch.nn.functional), used for the CPU/gloo config and as the numerics
  reference of the kernels.  There is no runtime fallback on GPU: the native
  extension is required there (`ops.require_native`).

Tensors are NHWC, conv weights HWIO, linear weights [in, out] (the layouts
the reference uses for its TF variables, /root/reference/mpipy.py:38-53).
"""

from __future__ import annotations

import dataclasses
from typing import Optional

import torch
import torch.nn.functional as F

from . import native, ptr, stream_handle


@dataclasses.dataclass
class Param:
    """A trainable tensor: a view of the flat param buffer plus the matching
    view of the flat grad buffer the backward kernels write into."""

    value: torch.Tensor
    grad_view: torch.Tensor
    # bf16 MFMA convs: weight copies laid out for the forward / the stride-1
    # dgrad, kept current by the owner's Bf16Weights.refresh()
    wtb: Optional[torch.Tensor] = None
    wtb_d: Optional[torch.Tensor] = None


class ConvWeightCopies:
    """Re-laid copies of a model's conv weights that the conv kernels read
    instead of the fp32 HWIO master weights, in one buffer.

    kind "bf16" (bf16 conv mode): every MFMA-family conv weight (C, K % 64 ==
    0) as the bf16 forward layout [tap][co][ci] (Param.wtb) and the bf16
    stride-1 dgrad layout, taps reversed (Param.wtb_d).
    kind "f32flip" (fp32 conv mode): every R x R (R > 1) conv weight with C, K
    % 32 == 0 as the fp32 stride-1 dgrad weights, taps reversed and ci / co
    transposed (Param.wtb_d; the tiled dgrad then skips its wflip launch).

    Kept current two ways: refresh() re-derives them all in ONE wcvt_batch
    launch (start of a run of steps, evaluation: any weight change made
    outside the step), and sgd() - the step's flat momentum SGD - writes them
    from the updated weights in the same launch (gops::sgd_wcvt), so a
    training step has no conversion launch of its own.  sgd() needs the flat
    parameter buffer (`flat`) the Params are views of."""

    def __init__(self, params, device: torch.device, flat: Optional[torch.Tensor] = None,
                 kind: str = "bf16"):
        C = native()
        if kind == "bf16":
            eligible = [p for p in params.values() if p.value.dim() == 4
                        and p.value.shape[2] % 64 == 0 and p.value.shape[3] % 64 == 0]
            modes, dt = (0, 1), torch.bfloat16
        elif kind == "f32flip":
            eligible = [p for p in params.values() if p.value.dim() == 4
                        and p.value.shape[0] == p.value.shape[1] and p.value.shape[0] > 1
                        and p.value.shape[2] % 32 == 0 and p.value.shape[3] % 32 == 0]
            modes, dt = (2,), torch.float32
        else:
            raise ValueError(kind)
        self.kind = kind
        self.buf = torch.empty(max(1, sum(len(modes) * p.value.numel() for p in eligible)),
                               dtype=dt, device=device)
        rows, off, blocks = [], 0, 0
        sgd_jobs, sblocks = [], 0
        for p in eligible:
            R, S, Ci, K = p.value.shape
            n = p.value.numel()
            outs = []
            for mode in modes:
                out = self.buf[off:off + n]
                off += n
                outs.append(out)
                rows.append([ptr(p.value), ptr(out), R * S, Ci, K, mode, blocks, 0])
                blocks += C.ops.wcvt_blocks(R * S, Ci, K)
            if kind == "bf16":
                p.wtb, p.wtb_d = outs
            else:
                p.wtb_d = outs[0]
            if flat is not None:
                woff = (p.value.data_ptr() - flat.data_ptr()) // 4
                o1 = ptr(outs[1]) if len(outs) > 1 else 0
                sgd_jobs.append([woff, ptr(outs[0]), o1, R * S, Ci, K, sblocks,
                                 0 if kind == "bf16" else 1])
                sblocks += C.ops.wcvt_blocks(R * S, Ci, K)
        self.njobs, self.nblocks = len(rows), blocks
        self.jobs = torch.tensor(rows if rows else [[0] * 8], dtype=torch.int64, device=device)
        self.flat = flat
        if flat is not None:
            # the float4 ranges of the flat buffer outside the eligible conv
            # weights (segments are 4-float aligned, parallel/flat.py)
            covered = sorted((j[0], j[0] + p.value.numel()) for j, p in zip(sgd_jobs, eligible))
            ranges, lo, rb = [], 0, 0
            for a, b in covered + [(flat.numel(), flat.numel())]:
                if a > lo:
                    assert lo % 4 == 0 and a % 4 == 0, "flat segments must be 4-float aligned"
                    n4 = (a - lo) // 4
                    nb = max(1, min(64, -(-n4 // 256)))
                    ranges.append([lo // 4, a // 4, rb, nb])
                    rb += nb
                lo = max(lo, b)
            self.sgd_njobs, self.sgd_conv_blocks = len(sgd_jobs), sblocks
            self.sgd_jobs = torch.tensor(sgd_jobs if sgd_jobs else [[0] * 8], dtype=torch.int64,
                                         device=device)
            self.nranges, self.range_blocks = len(ranges), rb
            self.ranges = torch.tensor(ranges if ranges else [[0] * 4], dtype=torch.int64,
                                       device=device)

    def refresh(self) -> None:
        if self.njobs:
            native().ops.wcvt_batch(ptr(self.jobs), self.njobs, self.nblocks, stream_handle())

    def sgd(self, grads: torch.Tensor, mom: torch.Tensor, momentum: float, gscale: float,
            lr: torch.Tensor, step: Optional[torch.Tensor]) -> None:
        """w = flat params: g' = gscale g; m = momentum m + g'; w -= lr m, and
        the copies of the updated conv weights (one launch)."""
        native().ops.sgd_wcvt(ptr(self.flat), ptr(grads), ptr(mom), momentum, gscale, 0.0,
                              ptr(lr), ptr(step), ptr(self.sgd_jobs), self.sgd_njobs,
                              self.sgd_conv_blocks, ptr(self.ranges), self.nranges,
                              self.range_blocks, stream_handle())


Bf16Weights = ConvWeightCopies  # (the bf16 kind)


def _empty(shape, like):
    return torch.empty(shape, dtype=like.dtype, device=like.device)


# MFMA operand precision of the tiled conv kernels: False = fp32 MFMA, True =
# operands converted to bf16 while staged into LDS (v_mfma_f32_32x32x16_bf16,
# fp32 accumulation; activations, BN and grads stay fp32).  Set by the engine
# (cfg.dtype); captured per op call, so a graph keeps the mode it was
# captured with.
_CONV_BF16 = False


def set_conv_bf16(on: bool) -> None:
    global _CONV_BF16
    _CONV_BF16 = bool(on)


# Gradient-ready hook: when set (parallel/overlap.py BucketedAllReduce), the
# backward of every op reports each parameter-gradient view it has finished
# writing, so gradient buckets can be all-reduced while backward continues.
_GRAD_HOOK = None
# True while an engine runs backward seeded with an exact 1.0 (its persistent
# ones scalar): the loss backward then returns dlogits as is, with no seed
# fill and no dlogits * g launch per step
_UNIT_SEED = False


# Oracle mode: every op takes its plain-PyTorch path (torch.nn.functional,
# autograd) even for GPU tensors - the GPU-resident numerics reference of the
# native kernels over whole training runs (GenericEngine oracle=True)
_ORACLE = False


class oracle_mode:
    """Context manager: the ops run their PyTorch definitions on any device."""

    def __enter__(self):
        global _ORACLE
        self._prev, _ORACLE = _ORACLE, True
        return self

    def __exit__(self, *exc):
        global _ORACLE
        _ORACLE = self._prev
        return False


def set_unit_loss_seed(on: bool) -> None:
    global _UNIT_SEED
    _UNIT_SEED = bool(on)



def set_grad_hook(fn) -> None:
    global _GRAD_HOOK
    _GRAD_HOOK = fn


def _grad_done(*views) -> None:
    if _GRAD_HOOK is not None:
        for v in views:
            if v is not None:
                _GRAD_HOOK(v)


# Producer-written bf16 copies: in bf16 conv mode the BatchNorm apply kernels
# also write a bf16 copy of their output (forward y, backward dx), attached to
# the fp32 tensor; a consuming conv reads it as its bf16 operand instead of
# running its own to_bf16 pass.  The copy is used only while the tensor is
# unmodified (same version counter and storage), else the conv converts.
def _attach_bf16(t: torch.Tensor, tb: torch.Tensor) -> None:
    t._mta_bf16 = (tb, t._version, t.data_ptr())


def _bf16_twin(t: torch.Tensor) -> Optional[torch.Tensor]:
    """The attached bf16 copy of t if it is still valid, else None."""
    a = getattr(t, "_mta_bf16", None)
    if a is not None and a[1] == t._version and a[2] == t.data_ptr() and t.is_contiguous():
        return a[0]
    return None


def _bf16_copy(t: torch.Tensor, s) -> torch.Tensor:
    if t.dtype == torch.bfloat16:  # already bf16 (a bf16-input BatchNorm's dX)
        return t.contiguous()
    a = getattr(t, "_mta_bf16", None)
    if a is not None and a[1] == t._version and a[2] == t.data_ptr() and t.is_contiguous():
        return a[0]
    tb = torch.empty(t.shape, dtype=torch.bfloat16, device=t.device)
    native().ops.to_bf16(ptr(t), ptr(tb), t.numel(), s)
    return tb


# BatchNorm statistics from the neighbouring convs, wired explicitly by the
# model (models/generic.py) through one BnLink per BatchNorm and step:
#   * forward: the conv producing the BatchNorm's input (conv2d(bn_out=L))
#     writes the channel-major partial sums of its output shifted by
#     L.shift (the BatchNorm's running mean) in its epilogue -> L.fwd; the
#     BatchNorm (batchnorm(link=L)) then skips its statistics pass;
#   * backward: the BatchNorm records what a dgrad needs for its backward
#     sums (bf16 input x, the bf16 twin of y for the ReLU mask, mean, rstd)
#     in L.bwd_src; the conv consuming the BatchNorm's output
#     (conv2d(bn_in=L)) passes it to its dgrad, whose epilogue writes the
#     sums of Sigma dY' and Sigma dY' x_hat -> L.bwd, and the BatchNorm
#     backward skips its statistics pass when the dY it receives IS that dX.
class BnLink:
    """Statistics hand-offs of one BatchNorm for one forward + backward (see
    above).  shift: the BatchNorm's running mean (the producer's epilogue
    shifts its sums by it); the other fields are filled by the ops."""

    __slots__ = ("shift", "fwd", "bwd_src", "bwd")

    def __init__(self, shift: Optional[torch.Tensor] = None):
        self.shift = shift
        self.fwd = None      # (partial table, rows): the producer's forward sums
        self.bwd_src = None  # (x, yb, mean, rstd, relu): set by the BatchNorm forward
        self.bwd = None      # (partial table, rows, dX): the consumer dgrad's sums


# A/B switches of the BatchNorm statistics epilogues (set by tests and labs
# through the setters below; production runs the defaults)
_BNB_EPILOGUE = True
BN_FWD_EPILOGUE = True
# fp32 conv mode: the tiled forward's epilogue / split-K reduction can write
# them too.  Off by default (set_bn_fwd_f32 turns it on): ResNet-18 fp32 B=32
# measured 6.655 / 6.666 ms on vs 6.641 / 6.646 off - the 64-row fp32 tiles
# give P = 2 x M / 64 partial rows, and the finalize's strided reads of that
# table cost what the skipped statistics pass saved
_BN_FWD_F32 = False
# observer of the BatchNorm backward route ("epilogue" | "pass"), for tests
_BN_ROUTE_HOOK = None


def set_bn_route_hook(fn) -> None:
    """fn(route) is called by every BatchNorm backward with the statistics
    route it took: "epilogue" (a dgrad wrote the sums) or "pass"."""
    global _BN_ROUTE_HOOK
    _BN_ROUTE_HOOK = fn


def set_bn_fwd_epilogue(on: bool) -> None:
    """Let bf16 conv epilogues write the BatchNorm forward statistics
    (default on; off = the BatchNorm's own statistics pass)."""
    global BN_FWD_EPILOGUE
    BN_FWD_EPILOGUE = bool(on)


def set_bn_fwd_f32(on: bool) -> None:
    """fp32 conv mode: let the tiled forward write the consuming BatchNorm's
    batch statistics (see _BN_FWD_F32)."""
    global _BN_FWD_F32
    _BN_FWD_F32 = bool(on)


def set_bn_bwd_epilogue(on: bool) -> None:
    """Let dgrad epilogues write the BatchNorm backward statistics (default
    on; off = the BatchNorm's own statistics pass, for A/B tests)."""
    global _BNB_EPILOGUE
    _BNB_EPILOGUE = bool(on)


def _bf16_out(like: torch.Tensor) -> Optional[torch.Tensor]:
    """A bf16 twin for a BN output when a bf16 conv can consume it."""
    if not _CONV_BF16 or like.shape[-1] % 64 != 0:
        return None
    return torch.empty(like.shape, dtype=torch.bfloat16, device=like.device)


# ------------------------------------------------------------ grad joins --
class GradJoin:
    """Fuses the gradient sum at a tensor read by two branches (a ResNet
    block input: conv1 and the shortcut) into a conv dgrad epilogue instead
    of autograd's separate add kernel.  The shortcut's backward `stash`es its
    gradient here and hands autograd None; the conv1 dgrad (`final`) adds the
    stash in its epilogue.  Autograd runs the shortcut first (it is created
    later in the forward, so has the higher sequence number); should the
    order ever flip, `stash` adds into the already-written dX in place, which
    is still before the consumer of that gradient runs (it waits for both
    edges)."""

    __slots__ = ("g", "out")

    def __init__(self):
        self.g: Optional[torch.Tensor] = None
        self.out: Optional[torch.Tensor] = None

    def stash(self, grad: torch.Tensor) -> None:
        if self.out is not None:
            self.out.add_(grad)
        else:
            self.g = grad

    def take(self) -> Optional[torch.Tensor]:
        g, self.g = self.g, None
        return g


# ------------------------------------------------------------------- conv --
class _ConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, shape, relu, gw, gb, ws, join=None, role=None, wtb=None,
                wtb_d=None, out_bf16=False, bn_out=None, bn_in=None):
        C = native()
        x = x.contiguous()
        ctx.bf16 = _CONV_BF16
        s = stream_handle()
        # bf16 family: the conv reads a bf16 copy of its input (half the
        # operand bytes of the fp32 tensor; kept for the filter gradient)
        xb = None
        if ctx.bf16 and C.ops.conv_bf16_ok(shape):
            xb = _bf16_copy(x, s)
        # out_bf16: the output is stored as bf16 (it feeds a bf16-input BatchNorm)
        oshape = (shape.N, shape.OH, shape.OW, shape.K)
        y = torch.empty(oshape, dtype=torch.bfloat16 if out_bf16 else x.dtype, device=x.device)
        part, rows = None, 0
        if bn_out is not None:  # the consuming BatchNorm's statistics
            # bf16 output: the bf16 family; fp32: the tiled forward (conv2d checks)
            rows = C.ops.conv_fwd_stats_rows(shape, bool(out_bf16))
            part = torch.empty(2 * shape.K * rows, dtype=torch.float32, device=x.device)
        # fp32: the stride-1 dgrad copy (f32flip) also feeds the forward's halo
        # kernel (conv_tiled.hip conv3f_kernel reads it with the taps reversed)
        C.ops.conv_fwd(shape, ptr(x), ptr(w), ptr(b), 0 if out_bf16 else ptr(y), relu, ptr(ws), s,
                       ctx.bf16, ptr(xb), ptr(wtb if ctx.bf16 else wtb_d),
                       ptr(y) if out_bf16 else 0, ptr(part), rows,
                       ptr(bn_out.shift) if part is not None else 0)
        if part is not None:
            bn_out.fwd = (part, rows)
        ctx.save_for_backward(x, w, y, xb)
        # x is a BatchNorm's output (bn_in): the dgrad can write that
        # BatchNorm's backward statistics (bf16 conv mode, bf16 BatchNorm input)
        ctx.bnb = bn_in if (ctx.bf16 and _BNB_EPILOGUE and bn_in is not None
                            and bn_in.bwd_src is not None) else None
        ctx.shape, ctx.relu, ctx.gw, ctx.gb, ctx.ws = shape, relu, gw, gb, ws
        ctx.has_b = b is not None
        ctx.join, ctx.role, ctx.wtb_d = join, role, wtb_d
        return y

    @staticmethod
    def backward(ctx, dy):
        C = native()
        x, w, y, xb = ctx.saved_tensors
        s = stream_handle()
        dy = dy.contiguous()
        if dy.dtype == torch.bfloat16:  # from a bf16-input BatchNorm: the bf16 kernels only
            dyb = dy
            C.ops.conv_bwd_filter(ctx.shape, ptr(x), 0, ptr(ctx.ws), ptr(ctx.gw), s, True,
                                  ptr(xb), ptr(dyb))
            _grad_done(ctx.gw)
            dx = None
            if ctx.needs_input_grad[0]:
                sh = ctx.shape
                dx = _empty((sh.N, sh.H, sh.W, sh.C), x)
                add = ctx.join.take() if ctx.role == "final" else None
                # the BatchNorm statistics need the final dX: not for a stashed
                # branch, nor a join whose other half is still to be added
                link = ctx.bnb if (ctx.role is None or (ctx.role == "final" and add is not None)) \
                    else None
                part, prow = None, 0
                if link is not None:
                    prow = C.ops.conv_bwd_data_stats_rows(sh)
                    if prow > 0:
                        part = torch.empty(2 * sh.C * prow, dtype=torch.float32, device=dx.device)
                if part is not None:
                    bx, byb, bmean, brstd, brelu = link.bwd_src
                    C.ops.conv_bwd_data(sh, 0, ptr(w), ptr(dx), ptr(ctx.ws), s, True, ptr(dyb),
                                        ptr(add), ptr(ctx.wtb_d), ptr(part), prow, ptr(bx),
                                        ptr(byb), ptr(bmean), ptr(brstd), brelu)
                    link.bwd = (part, prow, dx)
                else:
                    C.ops.conv_bwd_data(sh, 0, ptr(w), ptr(dx), ptr(ctx.ws), s, True, ptr(dyb),
                                        ptr(add), ptr(ctx.wtb_d))
                if ctx.role == "stash":
                    ctx.join.stash(dx)
                    dx = None
                elif ctx.role == "final" and add is None:
                    ctx.join.out = dx
            return (dx,) + (None,) * 14
        if ctx.relu:
            dym = torch.empty_like(dy)
            C.ops.relu_bwd(ptr(dy), ptr(y), ptr(dym), dy.numel(), s)
            dy = dym
        sh = ctx.shape
        dyb = None
        if xb is not None:  # one bf16 copy of dY feeds the filter grad and the dgrad
            dyb = _bf16_copy(dy, s)
        C.ops.conv_bwd_filter(sh, ptr(x), ptr(dy), ptr(ctx.ws), ptr(ctx.gw), s, ctx.bf16, ptr(xb),
                              ptr(dyb))
        if ctx.has_b:
            scratch = torch.empty(sh.K, device=dy.device, dtype=dy.dtype)
            C.ops.colsum2(ptr(dy), 0, sh.N * sh.OH * sh.OW, sh.K, ptr(ctx.gb), ptr(scratch), 0,
                          ptr(ctx.ws), s)
        _grad_done(ctx.gw, ctx.gb if ctx.has_b else None)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = _empty((sh.N, sh.H, sh.W, sh.C), dy)
            add = ctx.join.take() if ctx.role == "final" else None
            C.ops.conv_bwd_data(sh, ptr(dy), ptr(w), ptr(dx), ptr(ctx.ws), s, ctx.bf16, ptr(dyb),
                                ptr(add), ptr(ctx.wtb_d))
            if ctx.role == "stash":
                ctx.join.stash(dx)
                dx = None
            elif ctx.role == "final" and add is None:
                ctx.join.out = dx
        return (dx,) + (None,) * 14


class _ConvIm2colFn(torch.autograd.Function):
    """bf16 route for a thin-input conv whose input needs no gradient (the
    ResNet stem, 7x7 s2 over 3 channels): a bf16 im2col [N*OH*OW, kp] then a
    1x1 conv over kp channels on the bf16 family, forward and filter gradient.
    The im2col k order is per tap row (kh * seg + kw * C + ci, seg = S*C
    rounded up to 8), the weights are laid out to match.  Replaces the
    per-element gather engine (ResNet-18 B=32: 183 + 193 us per step on the
    stem)."""

    @staticmethod
    def forward(ctx, x, w, shape, gw, ws, kp, out_bf16=False, bn_out=None):
        C = native()
        x = x.contiguous()
        sh = shape
        sc, seg = sh.S * sh.C, _im2col_seg(sh)
        s = stream_handle()
        # weights in the im2col's k order (tap row kh at kh * seg, (kw, ci)
        # inside), written straight as the 1x1 conv's bf16 [K][kp] layout
        wtb = torch.empty(sh.K * kp, dtype=torch.bfloat16, device=x.device)
        if not out_bf16:
            C.ops.stem_weight_bf16(ptr(w), sh.R, sc, seg, kp, sh.K, ptr(wtb), s)
        s1 = C.ops.ConvShape(sh.N, sh.OH, sh.OW, kp, sh.K, 1, 1, 1, 0)
        y = torch.empty((sh.N, sh.OH, sh.OW, sh.K),
                        dtype=torch.bfloat16 if out_bf16 else x.dtype, device=x.device)
        # bf16 output (ResNet stem): the GEMM loaders gather the im2col on the fly
        # from the image (conv_bf16.hip StemLoader / StemWgLoader); else the
        # column matrix is materialised
        ctx.implicit = bool(out_bf16)
        ctx.s2d = None
        if ctx.implicit:
            part, rows = None, 0
            if bn_out is not None:  # the consuming BatchNorm's statistics
                rows = C.ops.conv_fwd_stem_stats_rows(s1)
                part = torch.empty(2 * sh.K * rows, dtype=torch.float32, device=x.device)
            shift = ptr(bn_out.shift) if part is not None else 0
            if _s2d_stem_ok(sh):
                # space-to-depth: the bf16 s2d image (saved for the filter
                # gradient) and the 8x8-extended filter, then the 4x4 conv
                si = _s2d_shape(sh)
                xs = torch.empty(sh.N * si.H * si.W * 16, dtype=torch.bfloat16, device=x.device)
                C.ops.s2d_stem_input(ptr(x), sh.N, sh.H, sh.W, sh.OH, sh.OW, ptr(xs), s)
                wt8 = torch.empty(sh.K * 256, dtype=torch.bfloat16, device=x.device)
                C.ops.s2d_stem_weight(ptr(w), sh.K, ptr(wt8), s)
                C.ops.conv_fwd_s2d_stem_bf16(si, ptr(xs), ptr(wt8), ptr(y), s, ptr(part), rows,
                                             shift)
                ctx.s2d = si
                ctx.save_for_backward(xs)
            else:
                C.ops.stem_weight_bf16(ptr(w), sh.R, sc, seg, kp, sh.K, ptr(wtb), s)
                C.ops.conv_fwd_stem_bf16(s1, sh, ptr(x), ptr(wtb), ptr(y), s, ptr(part), rows,
                                         shift)
                ctx.save_for_backward(x)
            if part is not None:
                bn_out.fwd = (part, rows)
        else:
            col = torch.empty((sh.N, sh.OH, sh.OW, kp), dtype=torch.bfloat16, device=x.device)
            C.ops.im2col_bf16(sh, ptr(x), kp, ptr(col), s)
            C.ops.conv_fwd(s1, 0, 0, 0, ptr(y), False, ptr(ws), s, True, ptr(col), ptr(wtb), 0)
            ctx.save_for_backward(col)
        ctx.s1, ctx.si, ctx.R, ctx.sc, ctx.seg, ctx.gw, ctx.ws = s1, sh, sh.R, sc, seg, gw, ws
        return y

    @staticmethod
    def backward(ctx, dy):
        C = native()
        (src,) = ctx.saved_tensors
        s1 = ctx.s1
        s = stream_handle()
        dy = dy.contiguous()
        dyb = _bf16_copy(dy, s)
        if ctx.s2d is not None:  # the 4x4 conv's filter gradient over the s2d image
            dw8 = torch.empty((256, s1.K), device=dy.device, dtype=torch.float32)
            C.ops.conv_bwd_filter_s2d_stem_bf16(ctx.s2d, ptr(src), ptr(dyb), ptr(ctx.ws), ptr(dw8),
                                                s)
            C.ops.s2d_stem_wgrad(ptr(dw8), s1.K, ptr(ctx.gw), s)
            _grad_done(ctx.gw)
            return None, None, None, None, None, None, None, None
        gpad = torch.empty((s1.C, s1.K), device=dy.device, dtype=torch.float32)
        if ctx.implicit:
            C.ops.conv_bwd_filter_stem_bf16(s1, ctx.si, ptr(src), ptr(dyb), ptr(ctx.ws), ptr(gpad),
                                            s)
        else:
            C.ops.conv_bwd_filter(s1, 0, 0, ptr(ctx.ws), ptr(gpad), s, True, ptr(src), ptr(dyb))
        C.ops.stem_wgrad(ptr(gpad), ctx.R, ctx.sc, ctx.seg, s1.K, ptr(ctx.gw), s)
        _grad_done(ctx.gw)
        return None, None, None, None, None, None, None, None


def _im2col_kp(sh, x: torch.Tensor, has_bias: bool, relu: bool) -> int:
    """kp (channels of the bf16 im2col route) for this conv, or 0 when the
    direct kernels take it: only bf16 mode, thin input (C % 64 != 0) that needs
    no gradient, K % 64 == 0, no bias / ReLU epilogue."""
    if not _CONV_BF16 or x.requires_grad or has_bias or relu or sh.C % 64 == 0:
        return 0
    rseg = sh.R * _im2col_seg(sh)
    if rseg < 64 or sh.K % 64 != 0:
        return 0
    return (rseg + 63) // 64 * 64


def _s2d_stem_ok(sh) -> bool:
    """The ResNet stem (7x7, stride 2, pad 3, 3 channels, K % 64 == 0) runs
    by space-to-depth (conv_bf16.hip conv_fwd_s2d_stem_bf16): a 4x4 stride-1
    conv over a bf16 image of 2x2 input blocks x 3 channels (+ 4 zero)."""
    return (sh.R == 7 and sh.S == 7 and sh.stride == 2 and sh.pad == 3 and sh.C == 3
            and sh.K % 64 == 0)


def _s2d_shape(sh):
    return native().ops.ConvShape(sh.N, sh.OH + 3, sh.OW + 3, 16, sh.K, 4, 4, 1, 0)


def _im2col_seg(sh) -> int:
    """Channels per tap row in the im2col layout: S*C rounded up to 8 (one
    16-byte bf16 store per 8)."""
    return (sh.S * sh.C + 7) // 8 * 8


class ConvWorkspace:
    """Split-K slab / reduction-partials workspace shared by the conv and BN
    kernels of all layers (they run in stream order).  Grown lazily.  A
    buffer is never released once handed out: captured hipGraphs keep its
    address, and a later, larger request (e.g. evaluation at a bigger batch
    between graph replays) must not let the allocator hand that memory to
    another tensor."""

    def __init__(self):
        self.t: Optional[torch.Tensor] = None
        self._retired = []

    def get(self, n: int, device) -> torch.Tensor:
        if self.t is None or self.t.numel() < n or self.t.device != device:
            if self.t is not None:
                self._retired.append(self.t)
            self.t = torch.empty(n, dtype=torch.float32, device=device)
        return self.t


_WS = ConvWorkspace()


def conv2d(x: torch.Tensor, w: Param, b: Optional[Param], stride: int = 1, pad: int = 0,
           relu: bool = False, join: Optional[GradJoin] = None,
           join_role: Optional[str] = None, out_bf16: bool = False,
           bn_out: Optional[BnLink] = None, bn_in: Optional[BnLink] = None) -> torch.Tensor:
    """x [N,H,W,C] NHWC, w [R,S,C,K] HWIO -> [N,OH,OW,K].  join / join_role
    ("stash" | "final"): fuse the gradient sum at x with another branch (see
    GradJoin).  out_bf16: store the output as bf16 when the bf16 conv family
    runs it (no bias / ReLU epilogue) - for a conv whose only consumer is
    `batchnorm`, which reads bf16 input.  bn_out (training): the BnLink of
    that BatchNorm - a bf16-output conv (or, in fp32 conv mode, the tiled fp32
    forward) then also writes the batch statistics in its epilogue (shifted by
    bn_out.shift) and the BatchNorm skips its statistics pass.  bn_in: the
    BnLink of the BatchNorm whose output x is - the dgrad then writes that
    BatchNorm's backward sums.  All GPU only, ignored on the CPU path."""
    N, H, W, Cin = x.shape
    R, S, _, K = w.value.shape
    if x.is_cuda and not _ORACLE:
        C = native()
        sh = C.ops.ConvShape(N, H, W, Cin, K, R, S, stride, pad)
        kp = _im2col_kp(sh, x, b is not None, relu)
        ob = bool(out_bf16 and _CONV_BF16 and b is None and not relu)
        if kp:
            s1 = C.ops.ConvShape(N, sh.OH, sh.OW, kp, K, 1, 1, 1, 0)
            nws = C.ops.conv_ws_floats(s1, False)
            if ob and _s2d_stem_ok(sh):
                nws = max(nws, C.ops.s2d_stem_ws_floats(_s2d_shape(sh)))
            ws = _WS.get(max(nws, 4), x.device)
            return _ConvIm2colFn.apply(x, w.value, sh, w.grad_view, ws, kp, ob,
                                       bn_out if ob else None)
        ob = ob and C.ops.conv_bf16_ok(sh)
        # fp32 conv mode: the tiled forward writes the statistics instead
        st32 = bool(bn_out is not None and not _CONV_BF16 and b is None and not relu and
                    _BN_FWD_F32 and C.ops.conv_fwd_tiled_ok(sh) and K % 64 == 0 and
                    256 % (K // 4) == 0)
        nws = max(C.ops.conv_ws_floats(sh, b is not None or relu),
                  C.ops.chan_reduce_ws_floats(N * sh.OH * sh.OW, K), 4)
        ws = _WS.get(nws, x.device)
        if join is not None and join_role == "final" and not C.ops.conv_bwd_data_join_ok(sh,
                                                                                         _CONV_BF16):
            raise ValueError("conv2d: no gradient-join epilogue for this conv shape")
        return _ConvFn.apply(x, w.value, None if b is None else b.value, sh, relu, w.grad_view,
                             None if b is None else b.grad_view, ws, join, join_role, w.wtb,
                             w.wtb_d, ob, bn_out if (ob or st32) else None, bn_in)
    y = F.conv2d(x.permute(0, 3, 1, 2), w.value.permute(3, 2, 0, 1),
                 None if b is None else b.value, stride=stride, padding=pad).permute(0, 2, 3, 1)
    return F.relu(y) if relu else y


class _LinearFn(torch.autograd.Function):
    """Fully connected layer on GPU through the in-tree VALU kernels
    (ops_generic.hip linear_fwd / linear_bwd): the FC layers of these models
    (LeNet-5 400-120-84-10 at batch 64, the ResNet-18 512 -> 10 head) are far
    below MFMA tile sizes.  Bias + ReLU run in the forward epilogue; backward is
    ONE launch (dW, db and dX block roles, ReLU mask applied on the fly) whose
    gradients land straight in the flat-buffer views."""

    @staticmethod
    def forward(ctx, x, w, b, relu, gw, gb):
        C = native()
        x = x.contiguous()
        M, K = x.shape
        N = w.shape[1]
        y = torch.empty((M, N), dtype=x.dtype, device=x.device)
        C.ops.linear_fwd(ptr(x), ptr(w), ptr(b), ptr(y), M, K, N, relu, stream_handle())
        ctx.save_for_backward(x, w, y if relu else None)
        ctx.relu, ctx.gw, ctx.gb = relu, gw, gb
        return y

    @staticmethod
    def backward(ctx, dy):
        C = native()
        x, w, y = ctx.saved_tensors
        dy = dy.contiguous()
        M, K = x.shape
        N = w.shape[1]
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        C.ops.linear_bwd(ptr(x), ptr(w), ptr(y), ptr(dy), ptr(ctx.gw), ptr(ctx.gb), ptr(dx), M, K,
                         N, ctx.relu, stream_handle())
        _grad_done(ctx.gw, ctx.gb)
        return dx, None, None, None, None, None


def linear(x: torch.Tensor, w: Param, b: Optional[Param], relu: bool = False) -> torch.Tensor:
    """x [N,in], w [in,out] -> [N,out]."""
    if x.is_cuda and not _ORACLE:
        return _LinearFn.apply(x, w.value, None if b is None else b.value, relu, w.grad_view,
                               None if b is None else b.grad_view)
    y = x @ w.value + (0 if b is None else b.value)
    return F.relu(y) if relu else y


# -------------------------------------------------------------- batchnorm --
class _BNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g, b, res, relu, gg, gb, rmean, rvar, momentum, eps, training,
                res_join=None, twin_only=False, link=None):
        C = native()
        x = x.contiguous()
        Cc = x.shape[-1]
        rows = x.numel() // Cc
        xb16 = x.dtype == torch.bfloat16  # a bf16-output conv's activations
        y = torch.empty(x.shape, dtype=torch.float32, device=x.device)
        mean = torch.empty(Cc, device=x.device)
        rstd = torch.empty(Cc, device=x.device)
        ws = _WS.get(max(C.ops.chan_reduce_ws_floats(rows, Cc), 4), x.device)
        yb = _bf16_out(y)
        # twin_only: the only consumer is a bf16 conv, so only the bf16 twin is
        # written (y's fp32 storage stays unwritten; the twin is attached)
        yf = None if (twin_only and yb is not None) else y
        # batch statistics, running-stat update and the fused apply, on device;
        # the statistics come from the producing conv's epilogue when it wrote them
        st = link.fwd if link is not None else None
        if st is not None:
            assert link.shift is rmean, "BnLink shift is not this BatchNorm's running mean"
            C.ops.bn_fwd_partials(ptr(st[0]), st[1], ptr(rmean), ptr(x), rows, Cc, ptr(g), ptr(b),
                                  ptr(res), ptr(yf), ptr(mean), ptr(rstd), eps, momentum, relu,
                                  ptr(rmean), ptr(rvar), stream_handle(), ptr(yb), xb16)
        else:
            C.ops.bn_fwd(ptr(x), rows, Cc, ptr(g), ptr(b), ptr(res), ptr(yf), ptr(mean), ptr(rstd),
                         ptr(ws), eps, momentum, relu, True, ptr(rmean), ptr(rvar),
                         stream_handle(), ptr(yb), xb16)
        if yb is not None:
            _attach_bf16(y, yb)
        if link is not None and xb16 and (yb is not None or not relu):
            link.bwd_src = (x, yb, mean, rstd, relu)
        ctx.link = link
        # the backward's ReLU mask reads the bf16 twin when there is one (same signs)
        ctx.yb16 = yb is not None
        ctx.save_for_backward(x, yb if yb is not None else y, mean, rstd, g)
        ctx.relu, ctx.gg, ctx.gb, ctx.has_res = relu, gg, gb, res is not None
        ctx.ws = ws
        ctx.res_join = res_join
        return y

    @staticmethod
    def backward(ctx, dy):
        C = native()
        x, y, mean, rstd, g = ctx.saved_tensors
        dy = dy.contiguous()
        Cc = x.shape[-1]
        rows = x.numel() // Cc
        xb16 = x.dtype == torch.bfloat16
        dres = torch.empty_like(dy) if ctx.has_res else None
        if xb16:
            # the gradient of a bf16 input is bf16 (autograd's dtype contract):
            # only the bf16 dX is written - the producing conv's backward reads
            # nothing else
            dx = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
            dxf, dxb = None, dx
        else:
            dx = torch.empty_like(dy)
            dxf, dxb = dx, _bf16_out(dx)
        st = None
        link = ctx.link
        if link is not None and link.bwd is not None and xb16 and (ctx.yb16 or not ctx.relu):
            part, prow, dxc = link.bwd
            # the sums are valid for exactly the dX that dgrad wrote
            if dxc.data_ptr() == dy.data_ptr() and dxc._version == dy._version:
                st = (part, prow)
        ctx.link = None
        if _BN_ROUTE_HOOK is not None:
            _BN_ROUTE_HOOK("epilogue" if st is not None else "pass")
        if st is not None:  # the dgrad producing dy wrote the sums (see above)
            C.ops.bn_bwd_partials(ptr(st[0]), st[1], ptr(x), ptr(dy), ptr(y), ptr(mean),
                                  ptr(rstd), ptr(g), rows, Cc, ctx.relu, ptr(ctx.gg), ptr(ctx.gb),
                                  ptr(dxf), ptr(dres), stream_handle(), ptr(dxb))
        else:
            C.ops.bn_bwd(ptr(x), ptr(dy), ptr(y), ptr(mean), ptr(rstd), ptr(g), rows, Cc,
                         ctx.relu, ptr(ctx.ws), ptr(ctx.gg), ptr(ctx.gb), ptr(dxf), ptr(dres),
                         stream_handle(), ptr(dxb), xb16, ctx.yb16)
        if dxf is not None and dxb is not None:
            _attach_bf16(dx, dxb)
        _grad_done(ctx.gg, ctx.gb)
        if dres is not None and ctx.res_join is not None:
            ctx.res_join.stash(dres)
            dres = None
        return dx, None, None, dres, None, None, None, None, None, None, None, None, None, None, None


def batchnorm(x: torch.Tensor, g: Param, b: Param, rmean: torch.Tensor, rvar: torch.Tensor,
              training: bool, relu: bool = False, residual: Optional[torch.Tensor] = None,
              momentum: float = 0.1, eps: float = 1e-5,
              res_join: Optional[GradJoin] = None, twin_only: bool = False,
              link: Optional[BnLink] = None) -> torch.Tensor:
    """BatchNorm over N,H,W of an NHWC tensor, optional fused residual + ReLU.
    res_join: the residual's gradient is stashed there (GradJoin) instead of
    returned to autograd.  twin_only: the output's only consumer is a bf16
    conv - write just its bf16 twin (bf16 conv mode; the returned fp32 tensor
    is not written).  link: this BatchNorm's BnLink (statistics from / for
    the neighbouring convs).  All GPU training only."""
    if x.is_cuda and not _ORACLE:
        res = None if residual is None else residual.contiguous()
        if training:
            return _BNFn.apply(x, g.value, b.value, res, relu, g.grad_view, b.grad_view, rmean,
                               rvar, momentum, eps, True, res_join, twin_only, link)
        C = native()
        y = torch.empty(x.shape, dtype=torch.float32, device=x.device)
        Cc = x.shape[-1]
        C.ops.bn_fwd(ptr(x.contiguous()), x.numel() // Cc, Cc, ptr(g.value), ptr(b.value),
                     ptr(res), ptr(y), 0, 0, 0, eps, momentum, relu, False, ptr(rmean),
                     ptr(rvar), stream_handle(), 0, x.dtype == torch.bfloat16)
        return y
    xn = x.permute(0, 3, 1, 2)
    y = F.batch_norm(xn, rmean, rvar, g.value, b.value, training, momentum, eps).permute(0, 2, 3, 1)
    if residual is not None:
        y = y + residual
    return F.relu(y) if relu else y


def softmax(logits: torch.Tensor) -> torch.Tensor:
    """Row softmax of [M, N] logits (no autograd): the prediction heads.
    Native kernel on GPU, torch on the CPU oracle path."""
    if not logits.is_cuda or _ORACLE:
        return torch.softmax(logits.float(), dim=1)
    x = logits.contiguous().float()
    y = torch.empty_like(x)
    native().ops.softmax_rows(ptr(x), ptr(y), x.shape[0], x.shape[1], stream_handle())
    return y


# ---------------------------------------------------------------- pooling --
class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, stride, pad):
        C = native()
        x = x.contiguous()
        N, H, W, Cc = x.shape
        sh = C.ops.PoolShape(N, H, W, Cc, k, stride, pad)
        y = _empty((N, sh.OH, sh.OW, Cc), x)
        s = stream_handle()
        xb = _bf16_twin(x)
        ctx.b8 = xb is not None and C.ops.maxpool_b16_ok(sh)
        if ctx.b8:
            # bf16 conv mode: pool the producer's bf16 twin (a twin-only BN
            # output), uint8 window-relative argmax, bf16 twin of the output
            arg = torch.empty((N, sh.OH, sh.OW, Cc), dtype=torch.uint8, device=x.device)
            yb = _bf16_out(y)
            C.ops.maxpool_fwd_b16(sh, ptr(xb), ptr(y), ptr(yb), ptr(arg), s)
            if yb is not None:
                _attach_bf16(y, yb)
        elif C.ops.maxpool_b16_ok(sh):
            # fp32: uint8 window-relative taps too (a quarter of the int32
            # argmax bytes; the backward's window-shared kernels take them)
            ctx.b8 = True
            arg = torch.empty((N, sh.OH, sh.OW, Cc), dtype=torch.uint8, device=x.device)
            C.ops.maxpool_fwd_u8(sh, ptr(x), ptr(y), ptr(arg), s)
        else:
            arg = torch.empty((N, sh.OH, sh.OW, Cc), dtype=torch.int32, device=x.device)
            C.ops.maxpool_fwd(sh, ptr(x), ptr(y), ptr(arg), s)
        ctx.save_for_backward(arg)
        ctx.sh, ctx.xshape = sh, x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        C = native()
        (arg,) = ctx.saved_tensors
        dx = _empty(ctx.xshape, dy)
        if ctx.b8:
            C.ops.maxpool_bwd_b8(ctx.sh, ptr(dy.contiguous()), ptr(arg), ptr(dx), stream_handle())
        else:
            C.ops.maxpool_bwd(ctx.sh, ptr(dy.contiguous()), ptr(arg), ptr(dx), stream_handle())
        return dx, None, None, None


def maxpool(x: torch.Tensor, k: int, stride: int, pad: int = 0) -> torch.Tensor:
    if x.is_cuda and not _ORACLE:
        return _MaxPoolFn.apply(x, k, stride, pad)
    return F.max_pool2d(x.permute(0, 3, 1, 2), k, stride, pad).permute(0, 2, 3, 1)


class _AvgPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        C = native()
        x = x.contiguous()
        N, H, W, Cc = x.shape
        y = torch.empty((N, Cc), dtype=x.dtype, device=x.device)
        C.ops.avgpool_fwd(ptr(x), ptr(y), N, H * W, Cc, stream_handle())
        ctx.xshape = x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        C = native()
        N, H, W, Cc = ctx.xshape
        dx = torch.empty(ctx.xshape, dtype=dy.dtype, device=dy.device)
        C.ops.avgpool_bwd(ptr(dy.contiguous()), ptr(dx), N, H * W, Cc, stream_handle())
        return dx


def global_avgpool(x: torch.Tensor) -> torch.Tensor:
    if x.is_cuda and not _ORACLE:
        return _AvgPoolFn.apply(x)
    return x.mean(dim=(1, 2))


# ------------------------------------------------------------------- loss --
class _XentFn(torch.autograd.Function):
    """Mean softmax cross-entropy in one launch (xent_mean_kernel writes the
    loss rows, dlogits and the mean) instead of xent + torch's mean."""

    @staticmethod
    def forward(ctx, logits, labels):
        C = native()
        logits = logits.contiguous()
        B, K = logits.shape
        loss_rows = torch.empty(B, device=logits.device)
        dlog = torch.empty_like(logits)
        mean = torch.empty((), device=logits.device)
        C.ops.xent_mean(ptr(logits), ptr(labels), B, K, ptr(loss_rows), ptr(dlog), ptr(mean), 0,
                        stream_handle())
        ctx.save_for_backward(dlog)
        return mean

    @staticmethod
    def backward(ctx, g):
        (dlog,) = ctx.saved_tensors
        if _UNIT_SEED:
            return dlog, None
        return dlog * g, None


def cross_entropy(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """mean softmax cross-entropy; labels int32 on GPU."""
    if logits.is_cuda and not _ORACLE:
        return _XentFn.apply(logits, labels.to(torch.int32))
    return F.cross_entropy(logits, labels.long())
