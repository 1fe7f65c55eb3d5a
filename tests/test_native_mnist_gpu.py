"""Numerics of the fused gfx950 MNIST kernels vs the plain-PyTorch fp32 oracle.

Each test runs the HIP path (`_C`, loaded in-tree) and compares against
`models/mnist_cnn.py` evaluated with torch ops in fp32 on the same inputs,
the same weights and the same dropout mask (utils/rng.py).
"""

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from mpi_tensorflow_amd import config as C
from mpi_tensorflow_amd.models import mnist_cnn as M
from mpi_tensorflow_amd.ops import native, ptr, stream_handle
from mpi_tensorflow_amd.runtime.mnist_engine import NativeMnistEngine, TorchMnistEngine
from mpi_tensorflow_amd.utils.data import synthetic_rows

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return (a - b).abs().max().item() / max(1e-6, b.abs().max().item())


@pytest.fixture(scope="module")
def data():
    x, y = synthetic_rows("train", 0, 1024)
    return x, y


def _engines(cuda_dev, data, **kw):
    x, y = data
    cfg = C.TrainConfig(graph=kw.pop("graph", False), **kw).validate()
    return NativeMnistEngine(cfg, x, y, cuda_dev), TorchMnistEngine(cfg, x, y, cuda_dev)


def test_conv_pool_forward_matches_oracle(cuda_dev, data):
    Cn = native()
    x, _ = data
    B = 96
    xd = torch.from_numpy(x[:B]).to(cuda_dev)
    g = torch.Generator().manual_seed(3)
    w1 = (torch.randn(5, 5, 1, 32, generator=g) * 0.2).to(cuda_dev)
    b1 = (torch.randn(32, generator=g) * 0.1).to(cuda_dev)
    w2 = (torch.randn(5, 5, 32, 64, generator=g) * 0.05).to(cuda_dev)
    b2 = (torch.randn(64, generator=g) * 0.1).to(cuda_dev)
    a1 = torch.empty(B, 14, 14, 32, device=cuda_dev)
    i1 = torch.empty(B, 14, 14, 32, dtype=torch.uint8, device=cuda_dev)
    a2 = torch.empty(B, 7, 7, 64, device=cuda_dev)
    i2 = torch.empty(B, 7, 7, 64, dtype=torch.uint8, device=cuda_dev)
    s = stream_handle()
    Cn.mnist.conv1_fwd(ptr(xd), 0, 0, B, ptr(w1), ptr(b1), ptr(a1), ptr(i1), s)
    w2t = torch.empty(25 * 64 * 32, device=cuda_dev)
    Cn.mnist.conv2_fwd(ptr(a1), B, ptr(w2), ptr(b2), ptr(a2), ptr(i2), ptr(w2t), s)
    torch.cuda.synchronize()
    xn = xd.permute(0, 3, 1, 2)
    z1 = F.conv2d(xn, w1.permute(3, 2, 0, 1), b1, padding=2)
    r1, ri1 = F.max_pool2d(F.relu(z1), 2, 2, return_indices=True)
    z2 = F.conv2d(r1, w2.permute(3, 2, 0, 1), b2, padding=2)
    r2 = F.max_pool2d(F.relu(z2), 2, 2)
    assert _rel(a1, r1.permute(0, 2, 3, 1)) < 1e-5
    assert _rel(a2, r2.permute(0, 2, 3, 1)) < 1e-5
    assert torch.equal(w2t.view(25, 64, 32), w2.view(25, 32, 64).transpose(1, 2))
    # argmax code of pool1 (where the ReLU output is positive the max is unique a.s.)
    iy = (ri1 // 28) % 2
    ix = (ri1 % 28) % 2
    code = (iy * 2 + ix).permute(0, 2, 3, 1).to(torch.uint8)
    pos = r1.permute(0, 2, 3, 1) > 0
    assert torch.equal(i1[pos], code[pos])


@pytest.mark.parametrize("step", [0, 3])
def test_fused_conv12_forward_matches_oracle(cuda_dev, data, step):
    """Train forward of conv1 + conv2 in one launch (conv1 recomputed into each
    conv2 block's halo): a1 / zero-bordered a1pf / idx1 / a2 / idx2 vs torch on
    the batch rows at the device-step offset."""
    Cn = native()
    x, _ = data
    B, n_local = 64, 512
    xd = torch.from_numpy(x[:n_local]).to(cuda_dev)
    g = torch.Generator().manual_seed(5)
    w1 = (torch.randn(5, 5, 1, 32, generator=g) * 0.2).to(cuda_dev)
    b1 = (torch.randn(32, generator=g) * 0.1).to(cuda_dev)
    w2 = (torch.randn(5, 5, 32, 64, generator=g) * 0.05).to(cuda_dev)
    b2 = (torch.randn(64, generator=g) * 0.1).to(cuda_dev)
    a1 = torch.empty(B, 14, 14, 32, device=cuda_dev)
    a1pf = torch.zeros(B, 18, 18, 32, device=cuda_dev)
    i1 = torch.empty(B, 14, 14, 32, dtype=torch.uint8, device=cuda_dev)
    a2 = torch.empty(B, 7, 7, 64, device=cuda_dev)
    i2 = torch.empty(B, 7, 7, 64, dtype=torch.uint8, device=cuda_dev)
    w2t = torch.empty(25 * 64 * 32, device=cuda_dev)
    st = torch.tensor([step], dtype=torch.int64, device=cuda_dev)
    Cn.mnist.conv12_fwd(ptr(xd), ptr(st), n_local, B, ptr(w1), ptr(b1), ptr(a1), ptr(a1pf),
                        ptr(i1), ptr(w2), ptr(b2), ptr(a2), ptr(i2), ptr(w2t), stream_handle())
    torch.cuda.synchronize()
    off = (step * B) % (n_local - B)
    # deterministic oracle: float64 on the CPU (a GPU oracle's convolutions
    # round differently from box to box and flip near-tied pooling argmaxes)
    c64 = lambda t: t.detach().cpu().double()  # noqa: E731
    xn = c64(xd[off:off + B]).permute(0, 3, 1, 2)
    z1 = F.relu(F.conv2d(xn, c64(w1).permute(3, 2, 0, 1), c64(b1), padding=2))
    r1 = F.max_pool2d(z1, 2, 2)
    z2 = F.relu(F.conv2d(r1, c64(w2).permute(3, 2, 0, 1), c64(b2), padding=2))
    r2 = F.max_pool2d(z2, 2, 2)
    r1h = r1.permute(0, 2, 3, 1)
    assert _rel(c64(a1), r1h) < 1e-5
    assert torch.equal(a1pf[:, 2:16, 2:16], a1)
    assert float(a1pf[:, :2].abs().sum() + a1pf[:, 16:].abs().sum()) == 0.0  # border untouched
    assert _rel(c64(a2), r2.permute(0, 2, 3, 1)) < 1e-5
    assert torch.equal(w2t.view(25, 64, 32), w2.view(25, 32, 64).transpose(1, 2))
    for idx, z in ((i1, z1), (i2, z2)):
        # the 2x2 windows, quadrant code 2 dy + dx; compare where the maximum is
        # positive and clear of the runner-up (an fp32 tie may go either way)
        Bn, Cc, H, W = z.shape
        win = z.view(Bn, Cc, H // 2, 2, W // 2, 2).permute(0, 2, 4, 1, 3, 5).reshape(
            Bn, H // 2, W // 2, Cc, 4)
        top = win.topk(2, dim=-1)
        code = top.indices[..., 0].to(torch.uint8)
        gap = top.values[..., 0] - top.values[..., 1]
        pos = (top.values[..., 0] > 0) & (gap > 1e-4 * top.values[..., 0].clamp(min=1.0))
        assert float(pos.float().mean()) > 0.3
        assert torch.equal(idx.cpu()[pos], code[pos])


@pytest.mark.parametrize("batch", [64, 96, 128])
def test_forward_backward_grads_match_oracle(cuda_dev, data, batch):
    """All grads of one native step vs the fp32 PyTorch oracle; batch 96
    exercises the partial K chunk of the fc1 dW role (K = batch)."""
    nat, ref = _engines(cuda_dev, data, batch_size=batch)
    nat.set_step(7)
    ref.set_step(7)
    nat.forward_backward_only()
    ref.forward_backward(7)
    torch.cuda.synchronize()
    assert abs(nat.bufs["loss_rows"].mean().item() - ref.last_loss) < 1e-4
    nv, rv = nat.layout.views(nat.grads), ref.layout.views(ref.grads)
    for s in nat.layout.specs:
        err = _rel(nv[s.name], rv[s.name])
        assert err < 2e-4, (s.name, err)


@pytest.mark.parametrize("algo,max_ties,tie_err", [("direct", 2, 5e-3), ("winograd", 4, 1e-2)])
def test_per_step_grads_along_native_trajectory(cuda_dev, data, algo, max_ties, tie_err):
    """Strict per-step check: at every step the native grads equal the oracle's
    grads evaluated at the NATIVE parameters (no chaotic accumulation).  The
    Winograd conv2 rounds differently from the oracle's direct sum (~1.4e-6
    relative, docs/ACCURACY.md) so max-pool near-ties re-route a gradient
    element somewhat more often than with the direct kernels."""
    nat, ref = _engines(cuda_dev, data, conv_algo=algo)
    ties = 0
    for step in range(12):
        ref.params.copy_(nat.params)
        ref.set_step(step)
        nat.forward_backward_only()
        ref.forward_backward(step)
        torch.cuda.synchronize()
        nv, rv = nat.layout.views(nat.grads), ref.layout.views(ref.grads)
        errs = {s.name: ((nv[s.name] - rv[s.name]).norm() / rv[s.name].norm()).item()
                for s in nat.layout.specs}
        print(step, {k: f"{v:.1e}" for k, v in errs.items()})
        # a max-pool near-tie (fp32 summation order) can re-route a single
        # element of dY2 / dA1, which shifts the conv grads (never the FC
        # grads) by ~1e-3 .. 5e-3 (Winograd rounding: up to 1e-2); everything
        # else must agree to fp32 rounding
        assert max(errs.values()) < tie_err, (step, errs)
        assert max(v for k, v in errs.items() if k.startswith("fc")) < 1e-4, (step, errs)
        if max(errs.values()) > 1e-4:
            ties += 1
        nat.train(1)
    assert ties <= max_ties, ties


@pytest.mark.parametrize("algo,bound", [("winograd", 7.5e-2), ("direct", 7.5e-2)])
def test_training_trajectory_matches_oracle(cuda_dev, data, algo, bound):
    """30 native steps vs the fp32 PyTorch oracle run on the CPU.  Both are
    deterministic (the oracle at a fixed thread count), so the drift is one
    reproducible number per conv2 algorithm: Winograd (the default) 6.69e-2,
    the direct 25-tap kernels 6.57e-2 (round 6; the GPU oracle's MIOpen
    convolutions moved it 3.6e-2 .. 5.24e-2 from box to box in round 4).  The
    two agree, so the drift is the max-pool / ReLU tie flips of fp32
    summation order compounding over the steps, not the Winograd arithmetic;
    the bound sits just above both: a native numerics change moves it.  The
    strict per-step check is test_per_step_grads_along_native_trajectory."""
    x, y = data
    cfg = C.TrainConfig(graph=False, conv_algo=algo).validate()
    nat = NativeMnistEngine(cfg, x, y, cuda_dev)
    nthreads = torch.get_num_threads()
    torch.set_num_threads(4)
    try:
        ref = TorchMnistEngine(cfg, x, y, torch.device("cpu"))
        p0 = ref.params.clone()
        losses_n, losses_r = [], []
        for _ in range(6):
            nat.train(5)
            ref.train(5)
            torch.cuda.synchronize()
            losses_n.append(nat.loss_value())
            losses_r.append(ref.loss_value())
    finally:
        torch.set_num_threads(nthreads)
    assert nat.step == ref.step == 30
    assert int(nat.step_dev.item()) == 30
    assert abs(nat.device_lr() - ref.lr(29)) < 1e-9
    # fp32 summation-order differences can flip a ReLU / max-pool tie and route
    # one element's gradient differently; over 30 steps that drift compounds,
    # so the trajectory is compared loosely (the strict check is per step)
    d = nat.params.cpu() - ref.params
    rel_upd = (d.norm() / (ref.params - p0).norm()).item()
    print(f"trajectory ({algo}): rel_update_err={rel_upd:.3e} losses native={losses_n} "
          f"ref={losses_r}")
    assert rel_upd < bound, rel_upd
    for a, b in zip(losses_n, losses_r):
        assert abs(a - b) < 2e-2 * max(1.0, abs(b))


def test_graph_replay_equals_eager(cuda_dev, data):
    eager, _ = _engines(cuda_dev, data)
    graphed, _ = _engines(cuda_dev, data, graph=True, graph_steps=4)
    eager.train(10)
    graphed.train(10)  # 2 replays of a 4-step graph + a 2-step graph
    torch.cuda.synchronize()
    assert torch.equal(eager.params, graphed.params)
    assert torch.equal(eager.mom, graphed.mom)


def test_eval_matches_oracle(cuda_dev, data):
    nat, ref = _engines(cuda_dev, data)
    nat.train(20)
    ref.params.copy_(nat.params)
    x, y = synthetic_rows("test", 0, 777)
    e_nat, logits = nat.evaluate(x, y, chunk=300, return_logits=True)
    e_ref = ref.evaluate(x, y)
    with torch.no_grad():
        lref = M.forward(ref.param_views(), torch.from_numpy(x).to(cuda_dev))
    assert _rel(logits, lref) < 1e-4
    assert abs(e_nat - e_ref) <= 100.0 * 2 / 777  # ties may flip at most a row or two


def test_sgd_kernel(cuda_dev):
    Cn = native()
    n = 4096
    g = torch.Generator().manual_seed(0)
    w = torch.randn(n, generator=g).to(cuda_dev)
    gr = torch.randn(n, generator=g).to(cuda_dev)
    m = torch.randn(n, generator=g).to(cuda_dev)
    lr = torch.tensor([0.05], device=cuda_dev)
    step = torch.zeros(1, dtype=torch.int64, device=cuda_dev)
    w0, m0 = w.clone(), m.clone()
    Cn.optim.sgd_momentum(ptr(w), ptr(gr), ptr(m), n, 1024, 5e-4, 0.9, 0.5, ptr(lr), 0.0,
                          ptr(step), stream_handle())
    torch.cuda.synchronize()
    ge = gr * 0.5
    ge[:1024] += 5e-4 * w0[:1024]
    me = 0.9 * m0 + ge
    we = w0 - 0.05 * me
    assert _rel(m, me) < 1e-6 and _rel(w, we) < 1e-6
    assert int(step.item()) == 1


def test_native_rccl_comm_and_graph_capture(cuda_dev, data):
    """World-size-1 RCCL communicator: dlopen of torch's librccl, unique-id
    bootstrap, all-reduce on a HIP stream, and the training step with both
    gradient buckets captured into a hipGraph (the 8-GPU path)."""
    from mpi_tensorflow_amd.parallel.comm import RcclDeviceComm
    from mpi_tensorflow_amd.parallel.dist import DistInfo

    comm = RcclDeviceComm(DistInfo())
    t = torch.arange(1000, dtype=torch.float32, device=cuda_dev)
    comm.all_reduce_(t)
    torch.cuda.synchronize()
    assert torch.equal(t, torch.arange(1000, dtype=torch.float32, device=cuda_dev))
    x, y = data
    cfg = C.TrainConfig(graph=True, graph_steps=3).validate()
    synced = NativeMnistEngine(cfg, x, y, cuda_dev, comm=comm, force_sync=True)
    plain = NativeMnistEngine(C.TrainConfig(graph=False).validate(), x, y, cuda_dev)
    assert synced.grad_sync and synced.comm_stream is not None
    synced.train(7)  # 2 replays of a captured 3-step graph (with RCCL) + a 1-step graph
    plain.train(7)
    torch.cuda.synchronize()
    assert torch.equal(synced.params, plain.params)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_fc_sgd_placements_bit_identical(cuda_dev, data, dtype):
    """Where the single-rank FC-bucket SGD runs - fp32: with the fc1 weight
    gradient formed inside it (fused dW1 tiles; fc1 backward runs without its
    dW1 role) in the final SGD launch (default) or as the tail of the
    Winograd bwd-data blocks; bf16: role blocks of the bwd-data launch
    (default) or the final launch - never changes the parameters or momenta
    (fp32 against the gradient-buffer path:
    test_native_rccl_comm_and_graph_capture)."""
    x, y = data
    runs = []
    for rounds in (-1, 0, 2):
        e = NativeMnistEngine(C.TrainConfig(graph=False, dtype=dtype).validate(), x, y, cuda_dev)
        e.exe.set_fc_sgd_rounds(rounds)
        e.train(7)
        runs.append(e)
    torch.cuda.synchronize()
    for e in runs[1:]:
        assert torch.equal(runs[0].params, e.params)
        assert torch.equal(runs[0].mom, e.mom)


def test_sync_schedule_autotune_with_emulated_ring(cuda_dev, data):
    """Startup autotune of the gradient-sync schedule (runtime/mnist_engine.py:
    tune_schedule) against an emulated 8-rank ring (csrc/collective.h EmuComm):
    every single-communicator schedule (buckets, serial, sharded, factors, defer) is
    captured and timed, the fastest is kept, and the trial steps are
    discarded: params, momentum and the step counter are restored."""
    from mpi_tensorflow_amd.parallel.comm import EmulatedDeviceComm

    x, y = data
    comm = EmulatedDeviceComm(8, lat_us=10.0, busbw_gbps=150.0, blocks=32)
    cfg = C.TrainConfig(graph=True, graph_steps=5).validate()
    eng = NativeMnistEngine(cfg, x, y, cuda_dev, comm=comm, force_sync=True)
    assert eng.sync_schedule == "buckets"  # default until tuned
    assert eng.comm2 is None  # auto never builds the two-communicator schedule
    p0 = eng.params.clone()
    ncand = len(eng._tune_candidates())  # buckets, serial, sharded, factors, defer
    n = eng.tune_schedule()
    assert ncand == 5 and n == ncand * 3 * 5 and eng.step == 0 and int(eng.step_dev.item()) == 0
    assert torch.equal(eng.params, p0)
    log = eng.tune_log
    assert set(log) == {"buckets", "serial", "sharded", "factors", "defer"}
    assert eng.sync_schedule == min(log, key=log.get)
    eng.train(7)
    torch.cuda.synchronize()
    assert torch.isfinite(eng.params).all()


@pytest.mark.parametrize("batch", [64, 96])
def test_fc1_forward_feature_major_matches_staged(cuda_dev, batch):
    """fc1 train forward over the feature-major a2t copy (LDS-free operands,
    8 split-K slabs) vs the LDS-staged kernel (14 slabs) and an fp64 matmul,
    with asymmetric data; and the Winograd conv2 forward's a2t equals the
    transpose of its a2 bit for bit."""
    Cn = native()
    k = Cn.mnist
    g = torch.Generator().manual_seed(21)
    a2 = torch.relu(torch.randn(batch, M.FC1_IN, generator=g)) * torch.rand(M.FC1_IN, generator=g)
    w = torch.randn(M.FC1_IN, M.FC1_OUT, generator=g) * 0.05 + 0.01
    a2d, a2td, wd = a2.to(cuda_dev), a2.t().contiguous().to(cuda_dev), w.to(cuda_dev)
    p_t = torch.full((k.fc1_part_floats(batch),), float("nan"), device=cuda_dev)
    p_s = torch.full_like(p_t, float("nan"))
    s = stream_handle()
    k.fc1_fwd_train_t(ptr(a2td), ptr(wd), batch, ptr(p_t), s)
    k.fc1_fwd_train(ptr(a2d), ptr(wd), batch, ptr(p_s), s)
    torch.cuda.synchronize()
    zt, zs = k.fc1_train_t_splits(), k.fc1_train_splits()
    ht = p_t[:zt * batch * M.FC1_OUT].view(zt, batch, M.FC1_OUT).sum(0).double().cpu()
    hs = p_s[:zs * batch * M.FC1_OUT].view(zs, batch, M.FC1_OUT).sum(0).double().cpu()
    ref = a2.double() @ w.double()
    assert torch.isfinite(ht).all()
    assert _rel(ht, ref) < 1e-6 and _rel(hs, ref) < 1e-6
    # the conv2 forward's feature-major copy
    x, y = synthetic_rows("train", 0, 4 * batch)
    e = NativeMnistEngine(C.TrainConfig(batch_size=batch, graph=False).validate(), x, y, cuda_dev,
                          fc1_feature_major=True)
    e.forward_backward_only()
    torch.cuda.synchronize()
    a2n = e.bufs["a2"].view(batch, M.FC1_IN)
    assert torch.equal(e.bufs["a2ft"].view(M.FC1_IN, batch), a2n.t())
