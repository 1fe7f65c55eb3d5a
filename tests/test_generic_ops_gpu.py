"""Numerics of the generic gfx950 layer kernels (csrc/kernels/ops_generic.hip)
vs plain PyTorch fp32, and of whole LeNet-5 / ResNet-18 training steps vs the
CPU oracle path."""

import dataclasses

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from mpi_tensorflow_amd import config as C
from mpi_tensorflow_amd.ops import functional as Fn

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / max(1e-12, b.float().norm())).item()


def _param(t):
    return Fn.Param(t.clone().requires_grad_(True), torch.zeros_like(t))


@pytest.mark.parametrize("N,H,W,Cin,K,R,stride,pad,relu,bias", [
    (4, 9, 7, 5, 6, 3, 1, 1, True, True),
    (4, 12, 12, 8, 16, 3, 2, 1, False, False),
    (2, 16, 16, 3, 64, 7, 2, 3, False, False),
    # fp32 gather-loader tiled forward (flattened (kh, kw, ci) K tiles, last one
    # partial): the stem with bias + ReLU and an M that is not a tile multiple
    (3, 20, 18, 3, 64, 7, 2, 3, True, True),
    (2, 15, 15, 5, 72, 5, 1, 2, False, False),   # K > 64: not a direct-kernel shape
    (3, 8, 8, 16, 32, 1, 2, 0, False, False),
    (5, 1, 1, 40, 70, 1, 1, 0, True, True),  # linear as a 1x1 conv
    # direct VALU forward (thin layers): the LeNet-5 conv shapes
    (4, 32, 32, 3, 6, 5, 1, 0, True, True),
    (4, 14, 14, 6, 16, 5, 1, 0, True, True),
    (3, 10, 11, 4, 8, 3, 1, 1, True, False),     # direct dgrad, K = 8
    # LDS-tiled family (conv_tiled.hip): ResNet-18 layer shapes, small batch
    (2, 14, 14, 64, 64, 3, 1, 1, False, False),
    (2, 14, 14, 64, 128, 3, 2, 1, False, False),  # stride-2 dgrad phases
    (2, 13, 13, 64, 128, 1, 2, 0, False, False),  # 1x1 s2 downsample, odd size
    (3, 7, 7, 256, 96, 3, 1, 1, True, True),
    (2, 9, 9, 32, 36, 5, 2, 2, False, True),
    (8, 1, 1, 512, 12, 1, 1, 0, False, True),     # FC 512 -> 12
    (10, 56, 56, 64, 64, 3, 1, 1, False, False),  # M >= 32768: 128-row tiles
])
def test_conv_fwd_bwd(cuda_dev, N, H, W, Cin, K, R, stride, pad, relu, bias):
    g = torch.Generator().manual_seed(0)
    x = torch.randn(N, H, W, Cin, generator=g)
    w = torch.randn(R, R, Cin, K, generator=g) * 0.2
    b = torch.randn(K, generator=g) * 0.1 if bias else None
    dy = torch.randn(N, (H + 2 * pad - R) // stride + 1, (W + 2 * pad - R) // stride + 1, K,
                     generator=g)
    # oracle
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True) if bias else None
    yr = F.conv2d(xr.permute(0, 3, 1, 2), wr.permute(3, 2, 0, 1), br, stride=stride,
                  padding=pad).permute(0, 2, 3, 1)
    if relu:
        yr = F.relu(yr)
    yr.backward(dy)
    # native
    xg = x.to(cuda_dev).requires_grad_(True)
    wp = _param(w.to(cuda_dev))
    bp = _param(b.to(cuda_dev)) if bias else None
    yg = Fn.conv2d(xg, wp, bp, stride, pad, relu)
    yg.backward(dy.to(cuda_dev))
    torch.cuda.synchronize()
    assert _rel(yg.cpu(), yr.detach()) < 1e-5
    assert _rel(xg.grad.cpu(), xr.grad) < 1e-5
    assert _rel(wp.grad_view.cpu(), wr.grad) < 1e-5
    if bias:
        assert _rel(bp.grad_view.cpu(), br.grad) < 1e-5


@pytest.mark.parametrize("relu,res", [(False, False), (True, False), (True, True)])
def test_batchnorm(cuda_dev, relu, res):
    g = torch.Generator().manual_seed(1)
    x = torch.randn(6, 5, 7, 24, generator=g) * 2 + 1
    r = torch.randn(6, 5, 7, 24, generator=g)
    gam = torch.rand(24, generator=g) + 0.5
    bet = torch.randn(24, generator=g)
    dy = torch.randn(6, 5, 7, 24, generator=g)
    xr = x.clone().requires_grad_(True)
    rr = r.clone().requires_grad_(True)
    gr, br = gam.clone().requires_grad_(True), bet.clone().requires_grad_(True)
    yr = F.batch_norm(xr.permute(0, 3, 1, 2), None, None, gr, br, True, 0.1, 1e-5).permute(0, 2, 3, 1)
    if res:
        yr = yr + rr
    if relu:
        yr = F.relu(yr)
    yr.backward(dy)
    xg = x.to(cuda_dev).requires_grad_(True)
    rg = r.to(cuda_dev).requires_grad_(True)
    gp, bp = _param(gam.to(cuda_dev)), _param(bet.to(cuda_dev))
    rm, rv = torch.zeros(24, device=cuda_dev), torch.ones(24, device=cuda_dev)
    yg = Fn.batchnorm(xg, gp, bp, rm, rv, True, relu, rg if res else None)
    yg.backward(dy.to(cuda_dev))
    torch.cuda.synchronize()
    assert _rel(yg.cpu(), yr.detach()) < 1e-5
    assert _rel(xg.grad.cpu(), xr.grad) < 1e-4
    assert _rel(gp.grad_view.cpu(), gr.grad) < 1e-4
    assert _rel(bp.grad_view.cpu(), br.grad) < 1e-5
    if res:
        assert _rel(rg.grad.cpu(), rr.grad) < 1e-6
    assert torch.allclose(rm.cpu(), 0.1 * x.mean(dim=(0, 1, 2)), atol=1e-5)


@pytest.mark.parametrize("C", [10, 16])  # scalar and float4 kernels
@pytest.mark.parametrize("k,stride,pad,H", [(2, 2, 0, 12), (3, 2, 1, 13)])
def test_maxpool(cuda_dev, k, stride, pad, H, C):
    g = torch.Generator().manual_seed(2)
    x = torch.randn(3, H, H, C, generator=g)
    xr = x.clone().requires_grad_(True)
    yr = F.max_pool2d(xr.permute(0, 3, 1, 2), k, stride, pad).permute(0, 2, 3, 1)
    dy = torch.randn(yr.shape, generator=g)
    yr.backward(dy)
    xg = x.to(cuda_dev).requires_grad_(True)
    yg = Fn.maxpool(xg, k, stride, pad)
    yg.backward(dy.to(cuda_dev))
    assert torch.equal(yg.cpu(), yr.detach())
    assert _rel(xg.grad.cpu(), xr.grad) < 1e-6


@pytest.mark.parametrize("C", [16, 64])
@pytest.mark.parametrize("H", [15, 14])  # C = 64: odd -> per-pixel, even -> 2x2-block bwd kernel
def test_maxpool_bf16_twin(cuda_dev, C, H):
    """bf16 conv mode: the pool reads the input's attached bf16 twin (a
    twin-only BN output, whose fp32 storage is garbage here on purpose),
    records uint8 window taps and gives its output a bf16 twin; values and
    gradients equal torch's pool of the bf16-rounded input."""
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, H, H, C, generator=g)
    xb = x.to(torch.bfloat16)
    xr = xb.float().clone().requires_grad_(True)
    yr = F.max_pool2d(xr.permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1)
    dy = torch.randn(yr.shape, generator=g)
    yr.backward(dy)
    xg = torch.full(x.shape, float("nan"), device=cuda_dev).requires_grad_(True)
    Fn._attach_bf16(xg, xb.to(cuda_dev))
    Fn.set_conv_bf16(True)
    yg = Fn.maxpool(xg, 3, 2, 1)
    yg.backward(dy.to(cuda_dev))
    torch.cuda.synchronize()
    assert torch.equal(yg.detach().cpu(), yr.detach())
    assert _rel(xg.grad.cpu(), xr.grad) < 1e-6
    tw = Fn._bf16_twin(yg)
    if C % 64 == 0:
        assert tw is not None and torch.equal(tw.float().cpu(), yr.detach())
    else:
        assert tw is None


def test_avgpool_and_xent(cuda_dev):
    g = torch.Generator().manual_seed(3)
    for C in (33, 512):  # per-(n, c) fallback, 32-channel x 8-group blocks
        x = torch.randn(4, 7, 7, C, generator=g)
        xg = x.to(cuda_dev).requires_grad_(True)
        y = Fn.global_avgpool(xg)
        y.sum().backward()
        assert _rel(y.cpu(), x.mean(dim=(1, 2))) < 1e-6
        assert torch.allclose(xg.grad.cpu(), torch.full_like(x, 1 / 49.0))
    logits = torch.randn(9, 13, generator=g)
    lab = torch.randint(0, 13, (9,), generator=g)
    lr_ = logits.clone().requires_grad_(True)
    F.cross_entropy(lr_, lab).backward()
    lg = logits.to(cuda_dev).requires_grad_(True)
    loss = Fn.cross_entropy(lg, lab.to(cuda_dev))
    loss.backward()
    assert abs(loss.item() - F.cross_entropy(logits, lab).item()) < 1e-5
    assert _rel(lg.grad.cpu(), lr_.grad) < 1e-5
    for B, K in ((64, 10), (257, 1000)):  # many blocks, K > 64 (lanes loop over classes)
        logits = torch.randn(B, K, generator=g) * 3
        lab = torch.randint(0, K, (B,), generator=g)
        lr_ = logits.clone().requires_grad_(True)
        F.cross_entropy(lr_, lab).backward()
        lg = logits.to(cuda_dev).requires_grad_(True)
        loss = Fn.cross_entropy(lg, lab.to(cuda_dev))
        loss.backward()
        assert abs(loss.item() - F.cross_entropy(logits, lab).item()) < 1e-4
        assert _rel(lg.grad.cpu(), lr_.grad) < 1e-5


@pytest.mark.parametrize("model,shape,B", [("lenet5", (32, 32, 3), 8), ("resnet18", (32, 32, 3), 4)])
def test_model_grads_native_vs_oracle(cuda_dev, model, shape, B):
    from mpi_tensorflow_amd.runtime.generic_engine import GenericEngine
    from mpi_tensorflow_amd.utils.data import synthetic_rows

    x, y = synthetic_rows("train", 0, 64, shape=shape)
    cfg = C.TrainConfig(model=model, batch_size=B, graph=False).validate()
    gpu = GenericEngine(cfg, x, y, cuda_dev)
    cpu = GenericEngine(C.TrainConfig(model=model, batch_size=B, device="cpu").validate(), x, y,
                        torch.device("cpu"))
    cpu.params.data.copy_(gpu.params.detach().cpu())
    gpu.train(1)
    cpu._step_cpu()
    torch.cuda.synchronize()
    assert abs(gpu.loss_value() - cpu.loss_value()) < 1e-4 * max(1.0, cpu.loss_value())
    gv, cv = gpu.layout.views(gpu.grads), cpu.layout.views(cpu.grads)
    for s in gpu.layout.specs:
        e = _rel(gv[s.name].cpu(), cv[s.name])
        assert e < 1e-3, (s.name, e)
    assert _rel(gpu.params.detach().cpu(), cpu.params.detach()) < 1e-4


def test_generic_graph_replay_equals_eager(cuda_dev):
    from mpi_tensorflow_amd.runtime.generic_engine import GenericEngine
    from mpi_tensorflow_amd.utils.data import synthetic_rows

    x, y = synthetic_rows("train", 0, 512, shape=(32, 32, 3))
    a = GenericEngine(C.TrainConfig(model="lenet5", graph=False).validate(), x, y, cuda_dev)
    b = GenericEngine(C.TrainConfig(model="lenet5", graph=True, graph_steps=4).validate(), x, y,
                      cuda_dev)
    a.train(13)
    b.train(13)  # 3 eager warm-up + 2 graph replays of 4 + 2 eager
    torch.cuda.synchronize()
    assert int(b.step_dev.item()) == 13
    assert _rel(b.params.detach(), a.params.detach()) < 1e-6


def test_generic_bucketed_allreduce_overlap(cuda_dev):
    """World-size-1 native RCCL: ResNet-18's gradient buckets are all-reduced
    on the comm stream in backward order, inside the captured hipGraph, and
    the result equals the unsynchronised run bit for bit."""
    from mpi_tensorflow_amd.parallel.comm import RcclDeviceComm
    from mpi_tensorflow_amd.parallel.dist import DistInfo
    from mpi_tensorflow_amd.runtime.generic_engine import GenericEngine
    from mpi_tensorflow_amd.utils.data import synthetic_rows

    comm = RcclDeviceComm(DistInfo())
    x, y = synthetic_rows("train", 0, 64, shape=(32, 32, 3))
    cfg = C.TrainConfig(model="resnet18", batch_size=8, graph=True, graph_steps=2).validate()
    synced = GenericEngine(cfg, x, y, cuda_dev, comm=comm, force_sync=True)
    plain = GenericEngine(C.TrainConfig(model="resnet18", batch_size=8, graph=False).validate(),
                          x, y, cuda_dev)
    assert synced.bucketer is not None
    synced.train(7)  # 3 eager warm-up steps + 2 replays of a 2-step graph
    plain.train(7)
    torch.cuda.synchronize()
    nb = len(synced.layout.buckets())
    assert nb == 6 and synced.bucketer.order == list(range(nb))  # backward completion order
    assert torch.equal(synced.params.detach(), plain.params.detach())


def test_generic_bucket_plan_autotune(cuda_dev):
    """bucket_plan="auto": the start-up tune times every distinct plan of
    parallel/overlap.py BUCKET_PLANS as captured graph replays on the native
    RCCL communicator, keeps one, and leaves no trace - the params, momentum,
    BatchNorm running statistics and step afterwards are those of before, so
    the tuned engine's training equals an untuned, unsynchronised run."""
    from mpi_tensorflow_amd.parallel.comm import RcclDeviceComm
    from mpi_tensorflow_amd.parallel.dist import DistInfo
    from mpi_tensorflow_amd.parallel.overlap import BUCKET_PLANS
    from mpi_tensorflow_amd.runtime.generic_engine import GenericEngine
    from mpi_tensorflow_amd.utils.data import synthetic_rows

    comm = RcclDeviceComm(DistInfo())
    x, y = synthetic_rows("train", 0, 64, shape=(32, 32, 3))
    cfg = C.TrainConfig(model="resnet18", dtype="bf16", batch_size=8, graph=True,
                        graph_steps=2).validate()
    tuned = GenericEngine(cfg, x, y, cuda_dev, comm=comm, force_sync=True)
    plain = GenericEngine(dataclasses.replace(cfg, graph=False), x, y, cuda_dev)
    before = tuned.params.detach().clone()
    steps = tuned.tune_schedule()
    torch.cuda.synchronize()
    assert steps > 0 and tuned.step == 0
    assert set(tuned.tune_log) == set(BUCKET_PLANS)
    assert all(v is not None and v > 0 for v in tuned.tune_log.values()), tuned.tune_log
    assert tuned.bucket_plan in BUCKET_PLANS
    assert min(tuned.tune_log.values()) == tuned.tune_log[tuned.bucket_plan]
    assert torch.equal(tuned.params.detach(), before)
    assert tuned.tune_schedule() == 0  # once
    tuned.train(7)
    plain.train(7)
    torch.cuda.synchronize()
    assert torch.equal(tuned.params.detach(), plain.params.detach())
    for k, (rm, rv) in plain.bn.items():
        assert torch.equal(tuned.bn[k][0], rm) and torch.equal(tuned.bn[k][1], rv)


@pytest.mark.parametrize("N,H,W,Cin,K,R,stride,pad", [
    (2, 14, 14, 64, 128, 3, 2, 1),
    (10, 56, 56, 64, 64, 3, 1, 1),
    (2, 9, 9, 3, 64, 7, 2, 3),  # stem-like: gather filter path
    (4, 7, 7, 512, 512, 3, 1, 1),  # layer4: split-K forward / backward-data
    (4, 14, 14, 128, 256, 1, 2, 0),  # 1x1 stride-2 downsample
    (8, 28, 28, 128, 128, 3, 1, 1),  # 128x128 tiles
    (3, 11, 13, 64, 192, 3, 1, 1),  # ragged M, non-square image
    (2, 14, 14, 256, 256, 3, 1, 1),  # layer3: all-taps wgrad, partial last row chunk
])
def test_conv_bf16_mfma(cuda_dev, N, H, W, Cin, K, R, stride, pad):
    """bf16-operand MFMA convolutions (fp32 accumulate) vs fp32 torch: relative
    error of bf16 input rounding (~2^-9 per operand)."""
    g = torch.Generator().manual_seed(7)
    x = torch.randn(N, H, W, Cin, generator=g)
    w = torch.randn(R, R, Cin, K, generator=g) * 0.1
    dy = torch.randn(N, (H + 2 * pad - R) // stride + 1, (W + 2 * pad - R) // stride + 1, K,
                     generator=g)
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    yr = F.conv2d(xr.permute(0, 3, 1, 2), wr.permute(3, 2, 0, 1), stride=stride,
                  padding=pad).permute(0, 2, 3, 1)
    yr.backward(dy)
    xg = x.to(cuda_dev).requires_grad_(True)
    wp = _param(w.to(cuda_dev))
    Fn.set_conv_bf16(True)
    try:
        yg = Fn.conv2d(xg, wp, None, stride, pad, False)
        yg.backward(dy.to(cuda_dev))
    finally:
        Fn.set_conv_bf16(False)
    torch.cuda.synchronize()
    assert _rel(yg.cpu(), yr.detach()) < 1e-2
    assert _rel(wp.grad_view.cpu(), wr.grad) < 1e-2
    if Cin % 4 == 0:
        assert _rel(xg.grad.cpu(), xr.grad) < 1e-2


def test_resnet18_bf16_trains(cuda_dev):
    from mpi_tensorflow_amd.runtime.generic_engine import GenericEngine
    from mpi_tensorflow_amd.utils.data import synthetic_rows

    x, y = synthetic_rows("train", 0, 256, shape=(32, 32, 3))
    tx, ty = synthetic_rows("test", 0, 128, shape=(32, 32, 3))
    eng = GenericEngine(C.TrainConfig(model="resnet18", batch_size=32, dtype="bf16",
                                      graph_steps=5).validate(), x, y, cuda_dev)
    e0 = eng.evaluate(tx, ty)
    eng.train(80)
    torch.cuda.synchronize()
    assert np.isfinite(eng.loss_value())
    assert eng.evaluate(tx, ty) < min(e0, 60.0)


def test_trainer_eval_between_graph_replays(cuda_dev):
    """Eval at a larger batch between captured-graph segments must not
    invalidate buffers the graphs still use (regression: LeNet NaN)."""
    from mpi_tensorflow_amd.runtime.trainer import Trainer

    cfg = C.TrainConfig(model="lenet5", max_steps=120, eval_every=30, graph_steps=10,
                        quiet=True).validate()
    s = Trainer(cfg).run()
    assert np.isfinite(s.final_loss), s
    assert s.final_test_error_global < 50.0, s


@pytest.mark.parametrize("out_bf16", [False, True])
@pytest.mark.parametrize("R,st,pad,K,kp,hw", [(7, 2, 3, 64, 192, (37, 41)),
                                              (7, 2, 3, 128, 192, (32, 48)),
                                              (5, 1, 2, 128, 128, (37, 41))])
def test_stem_conv_bf16_im2col_route(cuda_dev, R, st, pad, K, kp, hw, out_bf16):
    """bf16 mode: a thin-input conv whose input needs no gradient (ResNet stem,
    7x7 s2, 3 -> 64) runs as a 1x1 conv over its bf16 im2col on the bf16
    family - materialised (fp32 output), or, with bf16 output (the ResNet
    path), gathered on the fly by the GEMM loaders; the 7x7 s2 stem then runs
    by space-to-depth (a 4x4 s1 conv over the bf16 image of 2x2 blocks, odd and
    even image sizes).  Output and filter gradient vs fp32 torch within bf16
    operand rounding; the on-the-fly filter gradient equals the materialised
    one (bit for bit on the im2col loader; the s2d route sums in another
    order)."""
    from mpi_tensorflow_amd.ops import native

    g = torch.Generator().manual_seed(11)
    x = torch.randn(2, hw[0], hw[1], 3, generator=g)
    w = torch.randn(R, R, 3, K, generator=g) * 0.1
    wr = w.clone().requires_grad_(True)
    yr = F.conv2d(x.permute(0, 3, 1, 2), wr.permute(3, 2, 0, 1), stride=st,
                  padding=pad).permute(0, 2, 3, 1)
    dy = torch.randn(yr.shape, generator=g)
    yr.backward(dy)
    wp = _param(w.to(cuda_dev))
    xg = x.to(cuda_dev)
    sh = native().ops.ConvShape(2, hw[0], hw[1], 3, K, R, R, st, pad)
    Fn.set_conv_bf16(True)
    try:
        assert Fn._im2col_kp(sh, xg, False, False) == kp
        grads = []
        for ob in sorted({False, out_bf16}):
            wp.grad_view.zero_()
            yg = Fn.conv2d(xg, wp, None, st, pad, False, out_bf16=ob)
            assert yg.dtype == (torch.bfloat16 if ob else torch.float32)
            yg.backward(dy.to(cuda_dev).to(yg.dtype))
            torch.cuda.synchronize()
            grads.append(wp.grad_view.detach().clone())
    finally:
        Fn.set_conv_bf16(False)
    assert _rel(yg.detach().float().cpu(), yr.detach()) < 1e-2
    assert _rel(wp.grad_view.cpu(), wr.grad) < 1e-2
    if out_bf16 and Fn._s2d_stem_ok(sh):  # same bf16 products, another summation order
        assert _rel(grads[1].cpu(), grads[0].cpu()) < 1e-4
    elif out_bf16:  # same bf16 operands, same plan: the sums are identical
        assert torch.equal(grads[0], grads[1])


@pytest.mark.parametrize("hw", [(224, 224), (37, 41)])
def test_s2d_stem_preload_bit_identical(cuda_dev, hw):
    """The s2d stem forward with every K tile requested at once
    (S2dLoaderPre, default) stores the same tiles in the same LDS stages as
    the one-tile-ahead loader: outputs and BatchNorm partial rows bit for bit."""
    from mpi_tensorflow_amd.ops import native, ptr, stream_handle

    ops = native().ops
    g = torch.Generator().manual_seed(3)
    N, K = 4, 64
    x = torch.randn(N, hw[0], hw[1], 3, generator=g).to(cuda_dev)
    w = (torch.randn(7, 7, 3, K, generator=g) * 0.1).to(cuda_dev)
    sh = ops.ConvShape(N, hw[0], hw[1], 3, K, 7, 7, 2, 3)
    si = Fn._s2d_shape(sh)
    s = stream_handle()
    xs = torch.empty(N * si.H * si.W * 16, dtype=torch.bfloat16, device=cuda_dev)
    ops.s2d_stem_input(ptr(x), N, sh.H, sh.W, sh.OH, sh.OW, ptr(xs), s)
    wt8 = torch.empty(K * 256, dtype=torch.bfloat16, device=cuda_dev)
    ops.s2d_stem_weight(ptr(w), K, ptr(wt8), s)
    s1 = ops.ConvShape(N, sh.OH, sh.OW, 256, K, 1, 1, 1, 0)
    rows = ops.conv_fwd_stem_stats_rows(s1)
    shift = (torch.randn(K, generator=g) * 0.1).to(cuda_dev)
    outs = []
    try:
        for pre in (False, True):
            ops.s2d_stem_set_preload(pre)
            y = torch.empty(N, sh.OH, sh.OW, K, dtype=torch.bfloat16, device=cuda_dev)
            part = torch.empty(2 * K * rows, device=cuda_dev)
            ops.conv_fwd_s2d_stem_bf16(si, ptr(xs), ptr(wt8), ptr(y), s, ptr(part), rows,
                                       ptr(shift))
            torch.cuda.synchronize()
            outs.append((y, part))
    finally:
        ops.s2d_stem_set_preload(True)
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("N,H,W,C,K", [
    (8, 56, 56, 64, 64),    # 128-row tiles (ResNet layer 1 at B = 8), unsplit
    (2, 56, 56, 64, 64),    # 64-row tiles, 2 channel-chunk slices
    (4, 14, 14, 256, 256),  # split-K over the channel chunks
    (4, 28, 28, 128, 128),  # 128-row x 128-column tiles on the wide path
    (3, 7, 7, 512, 512),    # 16 chunks, partial last tile
    (2, 13, 9, 32, 64),     # odd image, one chunk
])
def test_fp32_halo_conv3x3_fwd_and_dgrad(cuda_dev, N, H, W, C, K):
    """fp32 3x3 / stride 1 / pad 1 convs on the halo kernel (conv_tiled.hip
    conv3f_kernel: forward reading the f32flip weight copy, taps reversed, and
    the stride-1 dgrad reading the HWIO weights, taps reversed) against a
    float64 torch reference and against the tiled kernels (TiledPlan halo_f32
    = False), through Fn.conv2d as the engine runs it (the filter gradient,
    tiled either way, checked alongside)."""
    from mpi_tensorflow_amd.ops import native

    ops = native().ops
    assert ops.conv3f_ok(ops.ConvShape(N, H, W, C, K, 3, 3, 1, 1))
    g = torch.Generator().manual_seed(7)
    x = torch.randn(N, H, W, C, generator=g)
    w = torch.randn(3, 3, C, K, generator=g) * (9 * C) ** -0.5
    dy = torch.randn(N, H, W, K, generator=g)
    xr = x.double().requires_grad_(True)
    wr = w.double().requires_grad_(True)
    yr = F.conv2d(xr.permute(0, 3, 1, 2), wr.permute(3, 2, 0, 1),
                  padding=1).permute(0, 2, 3, 1)
    yr.backward(dy.double())
    plan = ops.get_tiled_plan()
    outs = []
    try:
        # the halo kernel with 128-column tiles on 16-channel chunks (K % 128
        # == 0), with 64-column tiles on 32-channel chunks, each on 64- and
        # 128-row blocks, and the tiled kernels
        # (64-column tiles also on 16-channel chunks)
        # (and the small-footprint 64 x 64 variant: 288-row halo, 3-deep ring)
        for halo, wide, bm, ch, small in ((True, True, 64, 16, False), (True, True, 128, 16, False),
                                          (True, False, 64, 32, False), (True, False, 128, 32, False),
                                          (True, False, 64, 16, False), (True, False, 128, 16, False),
                                          (True, False, 0, 16, False), (True, False, 64, 16, True),
                                          (False, False, 64, 32, False)):
            p = ops.get_tiled_plan()
            p.halo_f32, p.halo_f32_wide, p.halo_f32_bm, p.halo_f32_ch = halo, wide, bm, ch
            p.halo_f32_small = small
            ops.set_tiled_plan(p)
            wp = _param(w.to(cuda_dev))
            Fn.ConvWeightCopies({"w": wp}, cuda_dev, kind="f32flip").refresh()
            xg = x.to(cuda_dev).requires_grad_(True)
            yg = Fn.conv2d(xg, wp, None, 1, 1, False)
            yg.backward(dy.to(cuda_dev))
            torch.cuda.synchronize()
            outs.append((yg.detach().cpu(), xg.grad.cpu(), wp.grad_view.detach().cpu().clone()))
    finally:
        ops.set_tiled_plan(plan)
    for yv, dx, dw in outs:
        assert _rel(yv.double(), yr.detach()) < 1e-5
        assert _rel(dx.double(), xr.grad) < 1e-5
        assert _rel(dw.double(), wr.grad) < 1e-5
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert _rel(a, b) < 1e-5


@pytest.mark.parametrize("N,H,C,K,R,stride,pad", [
    (8, 56, 64, 64, 3, 1, 1),   # 9 tiles x 256 slices (the 56x56 layer's plan)
    (4, 28, 64, 128, 3, 2, 1),  # stride 2, padded slice count
    (4, 28, 64, 128, 1, 2, 0),  # 1x1 stride 2
    (2, 40, 3, 64, 7, 2, 3),    # gather path (C = 3)
])
def test_fp32_filter_grad_xcd_slice_order(cuda_dev, N, H, C, K, R, stride, pad):
    """The fp32 filter gradient (conv_tiled.hip filter_kernel /
    filter_gather_kernel) with the XCD-grouped slice order and its zero padding
    slices (TiledPlan wg_xcd) and without, against a float64 torch reference."""
    from mpi_tensorflow_amd.ops import native

    ops = native().ops
    g = torch.Generator().manual_seed(11)
    x = torch.randn(N, H, H, C, generator=g)
    w = torch.randn(R, R, C, K, generator=g) * (R * R * C) ** -0.5
    xr = x.double()
    wr = w.double().requires_grad_(True)
    yr = F.conv2d(xr.permute(0, 3, 1, 2), wr.permute(3, 2, 0, 1), stride=stride,
                  padding=pad).permute(0, 2, 3, 1)
    dy = torch.randn(yr.shape, generator=g)
    yr.backward(dy.double())
    plan = ops.get_tiled_plan()
    outs = []
    try:
        # (and the 16-pixel K tiles of the 64 x 128 fp32 filter kernel)
        for xcd, bk16 in ((True, False), (False, False), (False, True)):
            p = ops.get_tiled_plan()
            p.wg_xcd, p.wg_bk16, p.wg_bk16_64 = xcd, bk16, bk16
            ops.set_tiled_plan(p)
            wp = _param(w.to(cuda_dev))
            yg = Fn.conv2d(x.to(cuda_dev), wp, None, stride, pad, False)
            yg.backward(dy.to(cuda_dev))
            torch.cuda.synchronize()
            outs.append(wp.grad_view.detach().cpu().clone())
    finally:
        ops.set_tiled_plan(plan)
    for dw in outs:
        assert _rel(dw.double(), wr.grad) < 1e-5
    assert _rel(outs[0], outs[1]) < 1e-6 and _rel(outs[1], outs[2]) < 1e-5


@pytest.mark.parametrize("N,H,C,K", [
    (4, 56, 64, 128),   # split over the output-channel chunks
    (2, 28, 128, 256),
    (3, 14, 256, 512),  # 7x7 dY grid, partial last tile
    (2, 10, 64, 32),    # 5x5 dY grid, two chunks
])
def test_fp32_dgrad3s2_halo(cuda_dev, N, H, C, K):
    """fp32 3x3 / stride 2 / pad 1 backward-data on the halo kernel
    (conv_tiled.hip dgrad3s2f_kernel: four parity-class accumulators over the
    staged dY halo, HWIO weights) and on the phase-split tiled kernel
    (TiledPlan halo_f32_s2 = False), against a float64 torch reference."""
    from mpi_tensorflow_amd.ops import native

    ops = native().ops
    g = torch.Generator().manual_seed(13)
    x = torch.randn(N, H, H, C, generator=g)
    w = torch.randn(3, 3, C, K, generator=g) * (9 * C) ** -0.5
    xr = x.double().requires_grad_(True)
    yr = F.conv2d(xr.permute(0, 3, 1, 2), w.double().permute(3, 2, 0, 1), stride=2,
                  padding=1).permute(0, 2, 3, 1)
    dy = torch.randn(yr.shape, generator=g)
    yr.backward(dy.double())
    plan = ops.get_tiled_plan()
    outs = []
    try:
        for halo in (True, False):
            p = ops.get_tiled_plan()
            p.halo_f32_s2 = halo
            ops.set_tiled_plan(p)
            wp = _param(w.to(cuda_dev))
            xg = x.to(cuda_dev).requires_grad_(True)
            yg = Fn.conv2d(xg, wp, None, 2, 1, False)
            yg.backward(dy.to(cuda_dev))
            torch.cuda.synchronize()
            outs.append(xg.grad.cpu())
    finally:
        ops.set_tiled_plan(plan)
    for dx in outs:
        assert _rel(dx.double(), xr.grad) < 1e-5
    assert _rel(outs[0], outs[1]) < 1e-5


def test_bn_bf16_twin_feeds_conv(cuda_dev):
    """bf16 mode: BatchNorm writes a bf16 twin of y (forward) and dx
    (backward); the consuming conv reads it instead of converting.  The result
    must be bit-identical to the convert-it-yourself path."""
    g = torch.Generator().manual_seed(5)
    x = torch.randn(4, 10, 10, 64, generator=g).to(cuda_dev)
    w = (torch.randn(3, 3, 64, 64, generator=g) * 0.05).to(cuda_dev)
    dy = torch.randn(4, 10, 10, 64, generator=g).to(cuda_dev)
    outs = []
    Fn.set_conv_bf16(True)
    try:
        for use_twin in (True, False):
            xg = x.clone().requires_grad_(True)
            gam, bet = _param(torch.ones(64, device=cuda_dev)), _param(torch.zeros(64, device=cuda_dev))
            wp = _param(w)
            rm, rv = torch.zeros(64, device=cuda_dev), torch.ones(64, device=cuda_dev)
            attach = Fn._attach_bf16
            if not use_twin:  # twins are written but never handed to the conv
                Fn._attach_bf16 = lambda t, tb: None
            try:
                h = Fn.batchnorm(xg, gam, bet, rm, rv, True, relu=True)
                assert hasattr(h, "_mta_bf16") == use_twin
                z = Fn.conv2d(h, wp, None, 1, 1, False)
                h2 = Fn.batchnorm(z, _param(torch.ones(64, device=cuda_dev)),
                                  _param(torch.zeros(64, device=cuda_dev)), rm.clone(), rv.clone(),
                                  True)
                h2.backward(dy)
            finally:
                Fn._attach_bf16 = attach
            torch.cuda.synchronize()
            outs.append((h2.detach().clone(), xg.grad.clone(), wp.grad_view.clone()))
    finally:
        Fn.set_conv_bf16(False)
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)


def test_batchnorm_large_mean_channels(cuda_dev):
    """Channels with mean ~1e3 and std ~1: the plain fp32 E[x^2] - mean^2
    variance loses every digit (mean^2 / var ~ 1e6 ~ 2^20 of a 2^24 mantissa);
    the shifted sums of bn.hip keep it within 1e-4 of an fp64 torch reference
    (output, running statistics and input gradient)."""
    g = torch.Generator().manual_seed(3)
    C = 32
    x = (torch.randn(8, 9, 11, C, generator=g, dtype=torch.float64) +
         1e3 * (1 + torch.rand(C, generator=g, dtype=torch.float64)))
    gam = torch.rand(C, generator=g, dtype=torch.float64) + 0.5
    bet = torch.randn(C, generator=g, dtype=torch.float64)
    dy = torch.randn(8, 9, 11, C, generator=g, dtype=torch.float64)
    xr = x.clone().requires_grad_(True)
    rm_ref, rv_ref = torch.zeros(C, dtype=torch.float64), torch.ones(C, dtype=torch.float64)
    yr = F.batch_norm(xr.permute(0, 3, 1, 2), rm_ref, rv_ref, gam, bet, True, 0.1,
                      1e-5).permute(0, 2, 3, 1)
    yr.backward(dy)
    xg = x.float().to(cuda_dev).requires_grad_(True)
    gp, bp = _param(gam.float().to(cuda_dev)), _param(bet.float().to(cuda_dev))
    rm, rv = torch.zeros(C, device=cuda_dev), torch.ones(C, device=cuda_dev)
    yg = Fn.batchnorm(xg, gp, bp, rm, rv, True, False, None)
    yg.backward(dy.float().to(cuda_dev))
    torch.cuda.synchronize()
    assert _rel(yg.cpu().double(), yr.detach()) < 1e-4
    assert _rel(rv.cpu().double(), rv_ref) < 1e-4
    assert _rel(rm.cpu().double(), rm_ref) < 1e-6
    assert _rel(xg.grad.cpu().double(), xr.grad) < 1e-3


@pytest.mark.parametrize("N,H,Cin,K,R,stride,pad,bf16", [
    (4, 14, 64, 64, 3, 1, 1, True),  # bf16 family, one K slab
    (4, 7, 512, 512, 3, 1, 1, True),  # bf16 family, split-K slab reduction
    (4, 14, 64, 128, 3, 2, 1, True),  # stride 2: tiled family
    (4, 14, 128, 64, 1, 2, 0, True),  # 1x1 stride 2: GEMM with the 2x2-expanding epilogue
    (4, 14, 64, 64, 3, 1, 1, False),  # fp32 tiled
    (2, 28, 128, 128, 3, 2, 1, False),
])
def test_conv_dgrad_gradient_join(cuda_dev, N, H, Cin, K, R, stride, pad, bf16):
    """The dgrad epilogue addend (Fn.GradJoin) equals dgrad + addend exactly
    (fp32 add of the same accumulator), on every family the ResNet joins use."""
    from mpi_tensorflow_amd.ops import native, ptr, stream_handle

    g = native().ops
    sh = g.ConvShape(N, H, H, Cin, K, R, R, stride, pad)
    assert g.conv_bwd_data_join_ok(sh, bf16)
    gen = torch.Generator().manual_seed(3)
    w = (torch.randn(R, R, Cin, K, generator=gen) * 0.1).to(cuda_dev)
    dy = torch.randn(N, sh.OH, sh.OW, K, generator=gen).to(cuda_dev)
    add = torch.randn(N, H, H, Cin, generator=gen).to(cuda_dev)
    ws = torch.empty(max(g.conv_ws_floats(sh, False), 4), device=cuda_dev)
    s = stream_handle()
    dx0 = torch.empty(N, H, H, Cin, device=cuda_dev)
    dx1 = torch.empty_like(dx0)
    dyb = dy.to(torch.bfloat16) if bf16 else None  # the pipelined bf16-operand kernel
    g.conv_bwd_data(sh, ptr(dy), ptr(w), ptr(dx0), ptr(ws), s, bf16, ptr(dyb))
    g.conv_bwd_data(sh, ptr(dy), ptr(w), ptr(dx1), ptr(ws), s, bf16, ptr(dyb), ptr(add))
    torch.cuda.synchronize()
    assert torch.equal(dx1, dx0 + add)


@pytest.mark.parametrize("M,K,N,relu", [(32, 512, 10, False), (64, 400, 120, True),
                                        (64, 84, 10, False), (5, 7, 200, True), (130, 33, 1, True)])
def test_linear_native_vs_torch(cuda_dev, M, K, N, relu):
    """Native FC forward (K split over lanes, LDS reduction) and the
    three-role backward vs fp32 torch."""
    gen = torch.Generator().manual_seed(11)
    x = torch.randn(M, K, generator=gen)
    w = torch.randn(K, N, generator=gen) * 0.1
    b = torch.randn(N, generator=gen)
    dy = torch.randn(M, N, generator=gen)
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    yr = xr @ wr + br
    yr = F.relu(yr) if relu else yr
    yr.backward(dy)
    xg = x.to(cuda_dev).requires_grad_(True)
    wp, bp = _param(w.to(cuda_dev)), _param(b.to(cuda_dev))
    yg = Fn.linear(xg, wp, bp, relu)
    yg.backward(dy.to(cuda_dev))
    torch.cuda.synchronize()
    assert _rel(yg.detach().cpu(), yr.detach()) < 1e-5
    assert _rel(wp.grad_view.cpu(), wr.grad) < 1e-5
    assert _rel(bp.grad_view.cpu(), br.grad) < 1e-5
    assert _rel(xg.grad.cpu(), xr.grad) < 1e-5


def test_bn_single_launch_reduction_repeatable(cuda_dev):
    """The one-launch BN statistics (last block sums the partial rows) on a
    ResNet layer-1 sized tensor: 20 back-to-back forward + backward passes
    give bit-identical results (a stale cross-XCD partial read would not),
    matching fp32 torch."""
    gen = torch.Generator().manual_seed(5)
    x = (torch.randn(32, 56, 56, 64, generator=gen) * 3 + 1).to(cuda_dev)
    dy = torch.randn(32, 56, 56, 64, generator=gen).to(cuda_dev)
    g = _param((torch.rand(64, generator=gen) + 0.5).to(cuda_dev))
    b = _param(torch.randn(64, generator=gen).to(cuda_dev))
    outs = []
    for _ in range(20):
        rm, rv = torch.zeros(64, device=cuda_dev), torch.ones(64, device=cuda_dev)
        xi = x.clone().requires_grad_(True)
        y = Fn.batchnorm(xi, g, b, rm, rv, True, relu=True)
        y.backward(dy)
        outs.append((y.detach().clone(), xi.grad.clone(), g.grad_view.clone(), rm.clone()))
    torch.cuda.synchronize()
    for o in outs[1:]:
        for a_, b_ in zip(o, outs[0]):
            assert torch.equal(a_, b_)
    # float64 reference: at 100k rows an fp32 reference's own rounding is ~1e-3
    xr = x.cpu().double().permute(0, 3, 1, 2).requires_grad_(True)
    yr = F.relu(F.batch_norm(xr, None, None, g.value.cpu().double(), b.value.cpu().double(), True,
                             0.1, 1e-5))
    yr.backward(dy.cpu().double().permute(0, 3, 1, 2))
    assert _rel(outs[0][0].cpu(), yr.detach().permute(0, 2, 3, 1)) < 1e-5
    # dX cancels (dy' - mean - xhat * mean) over 100k rows in fp32 (torch's own
    # fp32 backward is 2.3e-4 off the fp64 one here)
    assert _rel(outs[0][1].cpu(), xr.grad.permute(0, 2, 3, 1)) < 2e-3


@pytest.mark.parametrize("N,H,Cin,K,R,stride,pad", [
    (4, 14, 64, 64, 3, 1, 1),     # halo conv, unsplit
    (4, 7, 512, 512, 3, 1, 1),    # halo conv, split-K: bf16 written by the slab reduction
    (2, 14, 64, 128, 3, 2, 1),    # generic bf16 forward; stride-2 dgrad from bf16 dY (tiled)
    (2, 14, 64, 128, 1, 2, 0),    # 1x1 stride-2 downsample
    (2, 20, 3, 64, 7, 2, 3),      # stem: bf16 im2col route
])
def test_conv_bf16_output_and_bf16_grad(cuda_dev, N, H, Cin, K, R, stride, pad):
    """bf16-stored conv output (out_bf16, the ResNet bf16 path) and the
    backward fed a bf16 dY (what a bf16-input BatchNorm returns) vs fp32 torch."""
    g = torch.Generator().manual_seed(13)
    x = torch.randn(N, H, H, Cin, generator=g)
    w = torch.randn(R, R, Cin, K, generator=g) * 0.1
    OH = (H + 2 * pad - R) // stride + 1
    dy = torch.randn(N, OH, OH, K, generator=g)
    xr = x.clone().requires_grad_(Cin % 4 == 0)
    wr = w.clone().requires_grad_(True)
    yr = F.conv2d(xr.permute(0, 3, 1, 2), wr.permute(3, 2, 0, 1), stride=stride,
                  padding=pad).permute(0, 2, 3, 1)
    yr.backward(dy.to(torch.bfloat16).float())
    xg = x.to(cuda_dev).requires_grad_(Cin % 4 == 0)
    wp = _param(w.to(cuda_dev))
    Fn.set_conv_bf16(True)
    try:
        yg = Fn.conv2d(xg, wp, None, stride, pad, False, out_bf16=True)
        assert yg.dtype == torch.bfloat16
        yg.backward(dy.to(cuda_dev).to(torch.bfloat16))
    finally:
        Fn.set_conv_bf16(False)
    torch.cuda.synchronize()
    assert _rel(yg.float().cpu(), yr.detach()) < 1e-2
    assert _rel(wp.grad_view.cpu(), wr.grad) < 1e-2
    if Cin % 4 == 0:
        assert _rel(xg.grad.cpu(), xr.grad) < 1e-2


@pytest.mark.parametrize("N,H,Cin,K,R,stride,pad", [
    (4, 14, 64, 64, 3, 1, 1),     # halo conv, unsplit: statistics in its epilogue
    (4, 7, 512, 512, 3, 1, 1),    # halo conv, split-K: in the slab reduction
    (2, 14, 64, 128, 3, 2, 1),    # generic bf16 forward epilogue
    (2, 14, 64, 128, 1, 2, 0),    # 1x1 stride-2 downsample
    (2, 20, 3, 64, 7, 2, 3),      # stem: implicit-im2col epilogue
])
def test_conv_epilogue_bn_statistics(cuda_dev, N, H, Cin, K, R, stride, pad):
    """A bf16-output conv given the consuming BatchNorm's running mean
    (a BnLink) writes the batch statistics in its epilogue and the BatchNorm
    skips its own statistics pass: the BN output, the running statistics and
    the gradients match the two-pass BatchNorm on the same conv output."""
    g = torch.Generator().manual_seed(17)
    x = torch.randn(N, H, H, Cin, generator=g).to(cuda_dev)
    w = (torch.randn(R, R, Cin, K, generator=g) * 0.1).to(cuda_dev)
    gam = (torch.rand(K, generator=g) + 0.5).to(cuda_dev)
    bet = torch.randn(K, generator=g).to(cuda_dev)
    rm0 = (torch.randn(K, generator=g) * 0.3).to(cuda_dev)  # a nonzero shift
    OH = (H + 2 * pad - R) // stride + 1
    dy = torch.randn(N, OH, OH, K, generator=g).to(cuda_dev)
    out = []
    Fn.set_conv_bf16(True)
    try:
        for fused in (False, True):
            xi = x.clone().requires_grad_(Cin % 4 == 0)
            wp, gp, bp = _param(w), _param(gam), _param(bet)
            rm, rv = rm0.clone(), torch.ones(K, device=cuda_dev)
            lk = Fn.BnLink(rm) if fused else None
            y = Fn.conv2d(xi, wp, None, stride, pad, False, out_bf16=True, bn_out=lk)
            assert (lk is not None and lk.fwd is not None) == fused
            h = Fn.batchnorm(y, gp, bp, rm, rv, True, relu=True, link=lk)
            h.backward(dy)
            out.append((h.detach().clone(), rm.clone(), rv.clone(), wp.grad_view.clone(),
                        gp.grad_view.clone(), bp.grad_view.clone()))
    finally:
        Fn.set_conv_bf16(False)
    torch.cuda.synchronize()
    (h0, m0, v0, gw0, gg0, gb0), (h1, m1, v1, gw1, gg1, gb1) = out
    assert _rel(h1, h0) < 2e-5
    assert _rel(m1, m0) < 1e-5 and _rel(v1, v0) < 1e-5
    assert _rel(gw1, gw0) < 1e-4 and _rel(gg1, gg0) < 1e-4 and _rel(gb1, gb0) < 1e-5


@pytest.mark.parametrize("N,H,Cin,K,R,stride,pad", [
    (4, 14, 64, 64, 3, 1, 1),     # unsplit tiled forward: statistics in its epilogue
    (2, 7, 256, 512, 3, 1, 1),    # split-K: in the slab reduction
    (3, 9, 64, 128, 1, 2, 0),     # 1x1 stride-2 downsample, partial last tile
    (2, 20, 3, 64, 7, 2, 3),      # stem: gather-loader forward
])
def test_conv_epilogue_bn_statistics_fp32(cuda_dev, N, H, Cin, K, R, stride, pad):
    """fp32 conv mode: the tiled forward given the consuming BatchNorm's
    running mean writes the batch statistics in its epilogue (or split-K
    reduction) and the BatchNorm skips its statistics pass: output, running
    statistics and gradients match the two-pass BatchNorm on the same conv."""
    g = torch.Generator().manual_seed(19)
    x = torch.randn(N, H, H, Cin, generator=g).to(cuda_dev)
    w = (torch.randn(R, R, Cin, K, generator=g) * 0.1).to(cuda_dev)
    gam = (torch.rand(K, generator=g) + 0.5).to(cuda_dev)
    bet = torch.randn(K, generator=g).to(cuda_dev)
    rm0 = (torch.randn(K, generator=g) * 0.3).to(cuda_dev)  # a nonzero shift
    OH = (H + 2 * pad - R) // stride + 1
    dy = torch.randn(N, OH, OH, K, generator=g).to(cuda_dev)
    out = []
    Fn.set_bn_fwd_f32(True)
    try:
        for fused in (False, True):
            xi = x.clone().requires_grad_(Cin % 4 == 0)
            wp, gp, bp = _param(w), _param(gam), _param(bet)
            rm, rv = rm0.clone(), torch.ones(K, device=cuda_dev)
            lk = Fn.BnLink(rm) if fused else None
            y = Fn.conv2d(xi, wp, None, stride, pad, False, bn_out=lk)
            assert y.dtype == torch.float32
            assert (lk is not None and lk.fwd is not None) == fused
            h = Fn.batchnorm(y, gp, bp, rm, rv, True, relu=True, link=lk)
            h.backward(dy)
            out.append((h.detach().clone(), rm.clone(), rv.clone(), wp.grad_view.clone(),
                        gp.grad_view.clone(), bp.grad_view.clone()))
    finally:
        Fn.set_bn_fwd_f32(False)
    torch.cuda.synchronize()
    (h0, m0, v0, gw0, gg0, gb0), (h1, m1, v1, gw1, gg1, gb1) = out
    assert _rel(h1, h0) < 1e-5
    assert _rel(m1, m0) < 1e-6 and _rel(v1, v0) < 1e-5
    assert _rel(gw1, gw0) < 1e-5 and _rel(gg1, gg0) < 1e-5 and _rel(gb1, gb0) < 1e-6


@pytest.mark.parametrize("N,H,Cin,K,stride,relu", [
    (4, 14, 64, 64, 1, True),      # halo dgrad, unsplit: sums in its epilogue
    (4, 7, 512, 512, 1, False),    # halo dgrad, split-K: in the slab reduction
    (32, 56, 64, 128, 2, True),    # 3x3 stride-2 dgrad, unsplit
    (2, 28, 64, 128, 2, True),     # 3x3 stride-2 dgrad, split-K
])
def test_dgrad_epilogue_bn_backward_statistics(cuda_dev, N, H, Cin, K, stride, relu):
    """bf16 conv mode: the dgrad of a conv whose input is a BatchNorm output
    writes that BatchNorm's backward sums (sum dY', sum dY' xhat) in its
    epilogue (or its split-K reduction), and the BatchNorm backward skips its
    statistics pass: dX, dgamma and dbeta match the two-pass BatchNorm."""
    g = torch.Generator().manual_seed(31)
    x = (torch.randn(N, H, H, Cin, generator=g) * 2 + 0.5).to(torch.bfloat16).to(cuda_dev)
    w = (torch.randn(3, 3, Cin, K, generator=g) * 0.05).to(cuda_dev)
    gam = (torch.rand(Cin, generator=g) + 0.5).to(cuda_dev)
    bet = torch.randn(Cin, generator=g).to(cuda_dev)
    OH = (H + 2 - 3) // stride + 1
    dy = torch.randn(N, OH, OH, K, generator=g).to(torch.bfloat16).to(cuda_dev)
    out = []
    Fn.set_conv_bf16(True)
    try:
        routes = []
        Fn.set_bn_route_hook(routes.append)
        for fused in (False, True):
            Fn.set_bn_bwd_epilogue(fused)
            n0 = routes.count("epilogue")
            xi = x.clone().requires_grad_(True)
            gp, bp, wp = _param(gam), _param(bet), _param(w)
            rm, rv = torch.zeros(Cin, device=cuda_dev), torch.ones(Cin, device=cuda_dev)
            lk = Fn.BnLink()  # no forward hand-off here: the BatchNorm runs its pass
            h = Fn.batchnorm(xi, gp, bp, rm, rv, True, relu, link=lk)
            y = Fn.conv2d(h, wp, None, stride, 1, False, out_bf16=True, bn_in=lk)
            y.backward(dy)
            assert routes.count("epilogue") - n0 == (1 if fused else 0)
            out.append((xi.grad.float().clone(), gp.grad_view.clone(), bp.grad_view.clone(),
                        wp.grad_view.clone()))
    finally:
        Fn.set_bn_route_hook(None)
        Fn.set_bn_bwd_epilogue(True)
        Fn.set_conv_bf16(False)
    torch.cuda.synchronize()
    (dx0, gg0, gb0, gw0), (dx1, gg1, gb1, gw1) = out
    assert torch.equal(gw0, gw1)  # the filter gradient does not depend on the route
    nan = [bool(torch.isnan(t).any()) for t in (gg0, gb0, dx0, gg1, gb1, dx1)]
    assert not any(nan), f"NaN in (gg0, gb0, dx0, gg1, gb1, dx1): {nan}"
    assert _rel(gb1, gb0) < 1e-5 and _rel(gg1, gg0) < 1e-4
    assert _rel(dx1, dx0) < 4e-3  # dX is bf16: a few rounding flips


@pytest.mark.parametrize("relu,res", [(False, False), (True, True)])
def test_batchnorm_bf16_input(cuda_dev, relu, res):
    """BN over a bf16 input (a bf16-output conv's activations): statistics,
    apply and backward read the bf16 tensor; dX comes back bf16.  Reference:
    fp32 torch on the same bf16-rounded input."""
    g = torch.Generator().manual_seed(2)
    x = (torch.randn(8, 10, 10, 64, generator=g) * 2 + 0.5).to(torch.bfloat16)
    r = torch.randn(8, 10, 10, 64, generator=g)
    gam = torch.rand(64, generator=g) + 0.5
    bet = torch.randn(64, generator=g)
    dy = torch.randn(8, 10, 10, 64, generator=g)
    xr = x.float().requires_grad_(True)
    yr = F.batch_norm(xr.permute(0, 3, 1, 2), None, None, gam, bet, True, 0.1, 1e-5).permute(0, 2, 3, 1)
    if res:
        yr = yr + r
    if relu:
        yr = F.relu(yr)
    yr.backward(dy)
    xg = x.to(cuda_dev).requires_grad_(True)
    gp, bp = _param(gam.to(cuda_dev)), _param(bet.to(cuda_dev))
    rm, rv = torch.zeros(64, device=cuda_dev), torch.ones(64, device=cuda_dev)
    yg = Fn.batchnorm(xg, gp, bp, rm, rv, True, relu, r.to(cuda_dev) if res else None)
    assert yg.dtype == torch.float32
    yg.backward(dy.to(cuda_dev))
    torch.cuda.synchronize()
    assert xg.grad.dtype == torch.bfloat16
    assert _rel(yg.cpu(), yr.detach()) < 1e-5
    assert _rel(xg.grad.float().cpu(), xr.grad) < 1e-2  # bf16 rounding of dX
    assert _rel(gp.grad_view.cpu(), gam.grad if gam.grad is not None else
                (dy * (yr > 0 if relu else torch.ones_like(yr)) *
                 ((xr - xr.mean((0, 1, 2))) / (xr.var((0, 1, 2), unbiased=False) + 1e-5).sqrt())
                 ).sum((0, 1, 2)).detach()) < 1e-4
    assert torch.allclose(rm.cpu(), 0.1 * x.float().mean(dim=(0, 1, 2)), atol=1e-5)


def test_bn_twin_only_feeds_conv_identically(cuda_dev):
    """batchnorm(twin_only=True) writes only the bf16 twin of its output; a
    bf16 conv reading it gives bit-identical outputs and gradients to the
    full fp32 + twin version (and the ReLU mask comes from the twin)."""
    g = torch.Generator().manual_seed(21)
    x = torch.randn(4, 12, 12, 64, generator=g).to(torch.bfloat16).to(cuda_dev)
    w = (torch.randn(3, 3, 64, 64, generator=g) * 0.1).to(cuda_dev)
    gam, bet = (torch.rand(64, generator=g) + 0.5).to(cuda_dev), torch.randn(64, generator=g).to(cuda_dev)
    dy = torch.randn(4, 12, 12, 64, generator=g).to(torch.bfloat16).to(cuda_dev)
    out = []
    Fn.set_conv_bf16(True)
    try:
        for twin in (False, True):
            xi = x.clone().requires_grad_(True)
            gp, bp, wp = _param(gam), _param(bet), _param(w)
            rm, rv = torch.zeros(64, device=cuda_dev), torch.ones(64, device=cuda_dev)
            h = Fn.batchnorm(xi, gp, bp, rm, rv, True, True, twin_only=twin)
            y = Fn.conv2d(h, wp, None, 1, 1, False, out_bf16=True)
            y.backward(dy)
            out.append((y.detach().clone(), xi.grad.clone(), wp.grad_view.clone(),
                        gp.grad_view.clone(), bp.grad_view.clone()))
    finally:
        Fn.set_conv_bf16(False)
    torch.cuda.synchronize()
    for a_, b_ in zip(*out):
        assert torch.equal(a_, b_)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_resnet18_resume_restores_eval_gpu(cuda_dev, tmp_path, dtype):
    """GPU resume: ResNet-18 trained a few (graph-replayed) steps, saved with its
    BN running statistics, restored into a fresh engine: eval logits and error
    identical to before the save, and training continues identically."""
    from mpi_tensorflow_amd.runtime.generic_engine import GenericEngine
    from mpi_tensorflow_amd.utils import checkpoint as ck
    from mpi_tensorflow_amd.utils.data import synthetic_rows

    x, y = synthetic_rows("train", 0, 48, shape=(32, 32, 3))
    cfg = C.TrainConfig(model="resnet18", batch_size=8, dtype=dtype, graph=True,
                        graph_steps=2).validate()
    eng = GenericEngine(cfg, x, y, cuda_dev)
    eng.train(5)
    torch.cuda.synchronize()
    err0 = eng.evaluate(x[:16], y[:16])
    p = str(tmp_path / "r.npz")
    ck.save(p, eng.layout, eng.params, eng.mom, eng.step, meta={"model": "resnet18"},
            extra=eng.extra_state())
    e2 = GenericEngine(C.TrainConfig(model="resnet18", batch_size=8, dtype=dtype, graph=True,
                                     graph_steps=2, seed=7).validate(), x, y, cuda_dev)
    step, _ = ck.load(p, e2.layout, e2.params, e2.mom, extra=e2.extra_state(),
                      expect={"model": "resnet18"})
    e2.set_step(step)
    assert step == eng.step
    for k in eng.bn:
        assert torch.equal(eng.bn[k][0], e2.bn[k][0]) and torch.equal(eng.bn[k][1], e2.bn[k][1])
    assert e2.evaluate(x[:16], y[:16]) == err0
    eng.train(2)
    e2.train(2)
    torch.cuda.synchronize()
    assert torch.equal(eng.params.detach(), e2.params.detach())


def test_softmax_rows_native(cuda_dev):
    g = torch.Generator().manual_seed(4)
    x = torch.randn(37, 10, generator=g) * 5
    y = Fn.softmax(x.to(cuda_dev))
    torch.cuda.synchronize()
    assert _rel(y.cpu(), torch.softmax(x, 1)) < 1e-6


ROUTES = (False, True)


@pytest.mark.parametrize("shape,B", [((32, 32, 3), 32), ((224, 224, 3), 8)])
def test_resnet18_bn_backward_epilogue_matches_pass(cuda_dev, shape, B):
    """ResNet-18 bf16: one forward + backward with the BatchNorm backward sums
    written by the dgrad epilogues equals the same step with the BatchNorms'
    own statistics passes, parameter by parameter (same operands; only the
    summation order of the BN sums differs)."""
    from mpi_tensorflow_amd.runtime.generic_engine import GenericEngine
    from mpi_tensorflow_amd.utils.data import synthetic_rows

    x, y = synthetic_rows("train", 0, 4 * B, shape=shape)
    grads, counts = [], []
    routes = []
    Fn.set_bn_route_hook(routes.append)
    try:
        for on in ROUTES:
            Fn.set_bn_bwd_epilogue(on)
            eng = GenericEngine(C.TrainConfig(model="resnet18", batch_size=B, dtype="bf16",
                                              graph=False).validate(), x, y, cuda_dev)
            n0 = routes.count("epilogue")
            eng.forward_backward_gpu()
            torch.cuda.synchronize()
            counts.append(routes.count("epilogue") - n0)
            grads.append({k: v.clone() for k, v in eng.layout.views(eng.grads).items()})
    finally:
        Fn.set_bn_route_hook(None)
        Fn.set_bn_bwd_epilogue(True)
    assert all((c >= 12) == on for c, on in zip(counts, ROUTES)), counts
    errs = {k: _rel(grads[1][k], grads[0][k]) for k in grads[0]}
    # the head and the last block see the two routes' sums only through fp32
    # rounding (~1e-7); every BatchNorm further down the backward writes a bf16
    # dX, where such a difference flips the rounding of single elements (2^-8
    # relative), so the gap grows layer by layer (~1e-2 at the stem) without either route being wrong
    head = {k: v for k, v in errs.items() if k.startswith(("fc_", "l4b1n2", "l4b1c2", "l4b1n1"))}
    assert max(head.values()) < 1e-5, head
    worst = sorted(errs.items(), key=lambda kv: -kv[1])[:6]
    assert worst[0][1] < 3e-2, worst


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_sgd_writes_conv_weight_copies(cuda_dev, dtype):
    """ResNet-18: the step's fused SGD (gops::sgd_wcvt) updates every
    parameter bit-identically to the flat momentum SGD and writes the conv
    weights' re-laid copies - bf16: the MFMA forward / dgrad layouts; fp32:
    the flipped, ci / co-transposed stride-1 dgrad weights - exactly as the
    wcvt_batch re-derivation does (so no conversion launch is needed)."""
    from mpi_tensorflow_amd.ops import native, ptr, stream_handle
    from mpi_tensorflow_amd.runtime.generic_engine import GenericEngine
    from mpi_tensorflow_amd.utils.data import synthetic_rows

    x, y = synthetic_rows("train", 0, 16, shape=(32, 32, 3))
    eng = GenericEngine(C.TrainConfig(model="resnet18", batch_size=8, dtype=dtype,
                                      graph=False).validate(), x, y, cuda_dev)
    g = torch.Generator(device="cpu").manual_seed(5)
    grads = torch.randn(eng.layout.total, generator=g).to(cuda_dev)
    mom = torch.randn(eng.layout.total, generator=g).to(cuda_dev)
    lr = torch.tensor([0.0123], device=cuda_dev)
    step = torch.zeros(1, dtype=torch.int64, device=cuda_dev)
    w0 = eng.params.detach().clone()
    wc = eng.wcache
    assert wc is not None and wc.kind == ("bf16" if dtype == "bf16" else "f32flip")
    # reference: the flat SGD, then a full re-derivation of the copies
    m_ref = mom.clone()
    native().optim.sgd_momentum(ptr(eng.params), ptr(grads), ptr(m_ref), eng.layout.total, 0, 0.0,
                                0.9, 0.5, ptr(lr), 0.0, 0, stream_handle())
    wc.refresh()
    torch.cuda.synchronize()
    w_ref, buf_ref = eng.params.detach().clone(), wc.buf.clone()
    if dtype == "fp32":  # the copy's layout: W'[kh][kw][co][ci] = W[R-1-kh][S-1-kw][ci][co]
        p = eng.P["l1b0c2_w"]
        R, S, Ci, K = p.value.shape
        want = p.value.detach().flip(0).flip(1).permute(0, 1, 3, 2).contiguous()
        assert torch.equal(p.wtb_d.view(R, S, K, Ci), want)
    # fused
    eng.params.data.copy_(w0)
    wc.buf.zero_()
    wc.sgd(grads, mom, 0.9, 0.5, lr, step)
    torch.cuda.synchronize()
    assert int(step.item()) == 1
    assert torch.equal(eng.params.detach(), w_ref), "params differ from the flat SGD"
    assert torch.equal(mom, m_ref), "momentum differs from the flat SGD"
    assert torch.equal(wc.buf, buf_ref), "weight copies differ from wcvt_batch"
    assert wc.sgd_njobs > 0 and wc.nranges > 0


@pytest.mark.parametrize("N,H,C", [(4, 14, 64), (2, 28, 128), (8, 56, 64)])
def test_bn_finalize_fused_into_apply(cuda_dev, N, H, C):
    """The BatchNorm finalize (the partial-row reduction of the conv epilogue's
    statistics -> mean / rstd, or the backward sums) runs inside the apply
    launch behind a grid-wide barrier (bn.hip finalize_apply_kernel /
    finalize_bwd_apply_kernel): one launch per BatchNorm and direction instead
    of two.  Against the two-launch form on a conv -> BN(+ReLU) -> conv chain
    (forward statistics from the first conv's epilogue, backward sums from the
    second conv's dgrad epilogue): outputs, running statistics and every
    gradient agree (the same sums; only the few-row reduction order of the
    two-launch finalize64 differs), and no barrier spin timed out."""
    from mpi_tensorflow_amd.ops import native

    g = torch.Generator().manual_seed(23)
    x = (torch.randn(N, H, H, C, generator=g)).to(torch.bfloat16).to(cuda_dev)
    w1 = (torch.randn(3, 3, C, C, generator=g) * 0.05).to(cuda_dev)
    w2 = (torch.randn(3, 3, C, C, generator=g) * 0.05).to(cuda_dev)
    gam = (torch.rand(C, generator=g) + 0.5).to(cuda_dev)
    bet = torch.randn(C, generator=g).to(cuda_dev)
    rm0 = (torch.randn(C, generator=g) * 0.3).to(cuda_dev)
    dy = torch.randn(N, H, H, C, generator=g).to(torch.bfloat16).to(cuda_dev)
    ops = native().ops
    out = []
    Fn.set_conv_bf16(True)
    try:
        for fused, bpc in ((False, 2), (True, 2), (True, 8)):
            ops.bn_set_fused(fused)
            ops.bn_set_fused_blocks_per_cu(bpc)
            routes = []
            Fn.set_bn_route_hook(routes.append)
            p1, p2, gp, bp = _param(w1), _param(w2), _param(gam), _param(bet)
            rm, rv = rm0.clone(), torch.ones(C, device=cuda_dev)
            lk = Fn.BnLink(rm)
            y1 = Fn.conv2d(x, p1, None, 1, 1, False, out_bf16=True, bn_out=lk)
            assert lk.fwd is not None
            h = Fn.batchnorm(y1, gp, bp, rm, rv, True, relu=True, link=lk, twin_only=True)
            y2 = Fn.conv2d(h, p2, None, 1, 1, False, out_bf16=True, bn_in=lk)
            y2.backward(dy)
            torch.cuda.synchronize()
            assert routes == ["epilogue"], routes
            out.append((y2.detach().float().clone(), rm.clone(), rv.clone(), p1.grad_view.clone(),
                        p2.grad_view.clone(), gp.grad_view.clone(), bp.grad_view.clone()))
    finally:
        ops.bn_set_fused(False)
        ops.bn_set_fused_blocks_per_cu(2)
        Fn.set_bn_route_hook(None)
        Fn.set_conv_bf16(False)
    assert ops.bn_fused_error() == 0
    for a, b in zip(out[1], out[2]):  # the grid cap changes nothing but the launch
        assert torch.equal(a, b)
    for a, b in zip(out[0], out[1]):
        assert _rel(b, a) < 1e-4, (_rel(b, a))


@pytest.mark.gpu
def test_grid_barrier_cost(cuda_dev):
    """grid_sync.h's barrier at 224 blocks (the MNIST FC chain experiment's
    grid) and at 1-3 blocks a CU (the fused BatchNorm's): completes without a
    spin timeout; the cost per barrier is printed (PERF_NOTES round 6)."""
    from mpi_tensorflow_amd.ops import native

    ops = native().ops
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    for blocks in (224, cus, 2 * cus, 3 * cus):
        us = ops.gsync_barrier_us(blocks, 200)
        print(f"grid barrier: {blocks} blocks {us:.2f} us")
        assert 0 < us < 1000
    assert ops.bn_fused_error() == 0
