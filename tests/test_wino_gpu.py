"""Winograd F(2x2,5x5) conv2 kernels (csrc/kernels/wino.h, mnist.hip) vs the
plain PyTorch fp32 oracle of the reference's conv2 + ReLU + 2x2 max-pool
(/root/reference/mpipy.py:159-161).  The Winograd sums are fp32 throughout
but in another order than a direct 25-tap sum (error ~1e-6 relative,
scripts/wino_check.py), so values are compared at 2e-5 and argmax codes
wherever the pool window's maximum is unique by a clear margin."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from mpi_tensorflow_amd.ops import native, ptr, stream_handle
from mpi_tensorflow_amd.utils.data import synthetic_rows

pytestmark = pytest.mark.gpu

BT = np.array([[1, 1.5, -2, -1.5, 1, 0], [0, -1, -2.5, -0.5, 1, 0], [0, 1, 0.5, -2.5, 1, 0],
               [0, -0.5, -1, 0.5, 1, 0], [0, 2, -1, -2, 1, 0], [0, 1, 1.5, -2, -1.5, 1]])
G = np.array([[1, 0, 0, 0, 0], [-1 / 3] * 5, [1 / 3, -1 / 3, 1 / 3, -1 / 3, 1 / 3],
              [1 / 15, 2 / 15, 4 / 15, 8 / 15, 16 / 15], [-16 / 15, 8 / 15, -4 / 15, 2 / 15, -1 / 15],
              [0, 0, 0, 0, 1]])


def _rel(a, b):
    return (a - b).abs().max().item() / max(1e-6, b.abs().max().item())


def _weights(dev, seed=5):
    g = torch.Generator().manual_seed(seed)
    w1 = (torch.randn(5, 5, 1, 32, generator=g) * 0.2).to(dev)
    b1 = (torch.randn(32, generator=g) * 0.1).to(dev)
    w2 = (torch.randn(5, 5, 32, 64, generator=g) * 0.05).to(dev)
    b2 = (torch.randn(64, generator=g) * 0.1).to(dev)
    return w1, b1, w2, b2


def _pool_codes(z, r, idx, width):
    """argmax codes of the oracle pool where the window max is unique by 1e-4."""
    zz = z.permute(0, 2, 3, 1)  # NHWC pre-pool
    n, h, w, c = zz.shape
    win = zz.reshape(n, h // 2, 2, w // 2, 2, c).permute(0, 1, 3, 5, 2, 4).reshape(n, h // 2, w // 2, c, 4)
    top2 = win.topk(2, dim=-1).values
    clear = (top2[..., 0] - top2[..., 1]) > 1e-4 * (1 + top2[..., 0].abs())
    code = win.argmax(-1).to(torch.uint8)
    pos = (r.permute(0, 2, 3, 1) > 0) & clear
    return code, pos


def test_wino_filter_transform(cuda_dev):
    Cn = native()
    _, _, w2, _ = _weights(cuda_dev)
    U = torch.empty(36, 32, 64, device=cuda_dev)
    Ud = torch.empty(36, 64, 32, device=cuda_dev)
    Cn.mnist.conv2_wino_weights(ptr(w2), ptr(U), ptr(Ud), stream_handle())
    torch.cuda.synchronize()
    g = w2.double().cpu().numpy()  # [kh][kw][ci][co]
    want = np.einsum("ak,klio,bl->abio", G, g, G).reshape(36, 32, 64)
    # fragment order [p][ci/4][co/16][ci%4][co%16] -> [p][ci][co]
    got = U.view(36, 8, 4, 4, 16).permute(0, 1, 3, 2, 4).reshape(36, 32, 64).cpu().numpy()
    assert np.abs(got - want).max() < 1e-5 * np.abs(want).max()
    gr = g[::-1, ::-1].transpose(0, 1, 3, 2)  # rotated, [kh][kw][co][ci]
    want_d = np.einsum("ak,klio,bl->abio", G, gr, G).reshape(36, 64, 32)
    # [p][co/4][ci/16][co%4][ci%16] -> [p][co][ci]
    got_d = Ud.view(36, 16, 2, 4, 16).permute(0, 1, 3, 2, 4).reshape(36, 64, 32).cpu().numpy()
    assert np.abs(got_d - want_d).max() < 1e-5 * np.abs(want_d).max()


@pytest.mark.parametrize("B", [64, 96])
def test_wino_conv2_forward_matches_oracle(cuda_dev, B):
    Cn = native()
    x, _ = synthetic_rows("train", 0, B)
    xd = torch.from_numpy(x).to(cuda_dev)
    w1, b1, w2, b2 = _weights(cuda_dev)
    s = stream_handle()
    a1 = torch.empty(B, 14, 14, 32, device=cuda_dev)
    i1 = torch.empty(B, 14, 14, 32, dtype=torch.uint8, device=cuda_dev)
    Cn.mnist.conv1_fwd(ptr(xd), 0, 0, B, ptr(w1), ptr(b1), ptr(a1), ptr(i1), s)
    U = torch.empty(36 * 32 * 64, device=cuda_dev)
    Cn.mnist.conv2_wino_weights(ptr(w2), ptr(U), 0, s)
    a2 = torch.empty(B, 7, 7, 64, device=cuda_dev)
    i2 = torch.empty(B, 7, 7, 64, dtype=torch.uint8, device=cuda_dev)
    w2t = torch.empty(25 * 64 * 32, device=cuda_dev)
    Cn.mnist.conv2_fwd_wino(ptr(a1), B, ptr(w2), ptr(U), ptr(b2), ptr(a2), ptr(i2), ptr(w2t), s)
    torch.cuda.synchronize()
    r1 = a1.permute(0, 3, 1, 2)
    z2 = F.conv2d(r1.double(), w2.permute(3, 2, 0, 1).double(), b2.double(), padding=2)
    r2 = F.max_pool2d(F.relu(z2), 2, 2)
    assert _rel(a2.double(), r2.permute(0, 2, 3, 1)) < 2e-5
    assert torch.equal(w2t.view(25, 64, 32), w2.view(25, 32, 64).transpose(1, 2))
    code, pos = _pool_codes(z2, r2, i2, 14)
    assert pos.float().mean() > 0.2
    assert torch.equal(i2[pos], code[pos])


@pytest.mark.parametrize("step", [0, 3])
def test_wino_fused_conv12_forward_matches_oracle(cuda_dev, step):
    Cn = native()
    B, n_local = 64, 512
    x, _ = synthetic_rows("train", 0, n_local)
    xd = torch.from_numpy(x).to(cuda_dev)
    w1, b1, w2, b2 = _weights(cuda_dev, 7)
    a1 = torch.empty(B, 14, 14, 32, device=cuda_dev)
    a1pf = torch.zeros(B, 18, 18, 32, device=cuda_dev)
    i1 = torch.empty(B, 14, 14, 32, dtype=torch.uint8, device=cuda_dev)
    a2 = torch.empty(B, 7, 7, 64, device=cuda_dev)
    i2 = torch.empty(B, 7, 7, 64, dtype=torch.uint8, device=cuda_dev)
    w2t = torch.empty(25 * 64 * 32, device=cuda_dev)
    U = torch.empty(36 * 32 * 64, device=cuda_dev)
    st = torch.tensor([step], dtype=torch.int64, device=cuda_dev)
    s = stream_handle()
    Cn.mnist.conv2_wino_weights(ptr(w2), ptr(U), 0, s)
    Cn.mnist.conv12_fwd_wino(ptr(xd), ptr(st), n_local, B, ptr(w1), ptr(b1), ptr(a1), ptr(a1pf),
                             ptr(i1), ptr(w2), ptr(U), ptr(b2), ptr(a2), ptr(i2), ptr(w2t), s)
    torch.cuda.synchronize()
    off = (step * B) % (n_local - B)
    xn = xd[off:off + B].permute(0, 3, 1, 2).double()
    z1 = F.conv2d(xn, w1.permute(3, 2, 0, 1).double(), b1.double(), padding=2)
    r1 = F.max_pool2d(F.relu(z1), 2, 2)
    assert _rel(a1.double(), r1.permute(0, 2, 3, 1)) < 1e-5
    assert torch.equal(a1pf[:, 2:16, 2:16], a1)
    # the fused conv1 (its tiles spread over all 8 waves) equals the standalone
    # conv1 kernel bit for bit (each tile's K order is the same)
    a1s = torch.empty_like(a1)
    i1s = torch.empty_like(i1)
    Cn.mnist.conv1_fwd(ptr(xd), ptr(st), n_local, B, ptr(w1), ptr(b1), ptr(a1s), ptr(i1s), s, 0)
    torch.cuda.synchronize()
    assert torch.equal(a1s, a1) and torch.equal(i1s, i1)
    z2 = F.conv2d(a1.permute(0, 3, 1, 2).double(), w2.permute(3, 2, 0, 1).double(), b2.double(),
                  padding=2)
    r2 = F.max_pool2d(F.relu(z2), 2, 2)
    assert _rel(a2.double(), r2.permute(0, 2, 3, 1)) < 2e-5
    code, pos = _pool_codes(z2, r2, i2, 14)
    assert torch.equal(i2[pos], code[pos])


@pytest.mark.parametrize("B,dense", [(64, False), (96, False), (64, True)])
def test_wino_conv2_bwd_data_matches_oracle(cuda_dev, B, dense):
    """dA1 = conv2 backward-data of a sparse (pool-scattered, as fc1 bwd writes
    it) or dense dY2, masked by a1 > 0, vs torch autograd in fp64 (the dense
    case puts nonzeros on every border pixel the zero padding meets)."""
    Cn = native()
    g = torch.Generator().manual_seed(11)
    _, _, w2, _ = _weights(cuda_dev)
    a1 = torch.relu(torch.randn(B, 14, 14, 32, generator=g)).to(cuda_dev)
    # pre-pool gradient: one nonzero per 2x2 window (the argmax), as fc1 bwd writes it
    dpool = torch.randn(B, 7, 7, 64, generator=g)
    q = torch.randint(0, 4, (B, 7, 7, 64), generator=g)
    dy2 = torch.zeros(B, 14, 14, 64)
    for k in range(4):
        dy2[:, k >> 1::2, k & 1::2, :] = torch.where(q == k, dpool, torch.zeros(()))
    if dense:
        dy2 = torch.randn(B, 14, 14, 64, generator=g)
    dy2 = dy2.to(cuda_dev)
    Ud = torch.empty(36 * 64 * 32, device=cuda_dev)
    U = torch.empty(36 * 32 * 64, device=cuda_dev)
    s = stream_handle()
    Cn.mnist.conv2_wino_weights(ptr(w2), ptr(U), ptr(Ud), s)
    da1m = torch.full((B, 14, 14, 32), float("nan"), device=cuda_dev)
    Cn.mnist.conv2_bwd_data_wino(ptr(dy2), ptr(Ud), ptr(a1), B, ptr(da1m), s)
    torch.cuda.synchronize()
    x = a1.permute(0, 3, 1, 2).double().requires_grad_(True)
    z = F.conv2d(x, w2.permute(3, 2, 0, 1).double(), padding=2)
    z.backward(dy2.permute(0, 3, 1, 2).double())
    want = (x.grad * (x > 0)).permute(0, 2, 3, 1)
    assert torch.isfinite(da1m).all()
    assert _rel(da1m.double(), want) < 2e-5
    assert float(da1m[a1 <= 0].abs().sum()) == 0.0


def test_sgd_writes_current_winograd_filters(cuda_dev):
    """Single-rank steps take U / Ud from the previous step's SGD launch
    (sgd_finalize, per-input-channel blocks): after a few eager and replayed
    steps they must equal a fresh transform of the current conv2 weights, and
    the conv2 bias / conv1 parameters must have been updated normally."""
    from mpi_tensorflow_amd import config as C
    from mpi_tensorflow_amd.runtime.mnist_engine import NativeMnistEngine

    Cn = native()
    x, y = synthetic_rows("train", 0, 1024)
    for graph in (False, True):
        cfg = C.TrainConfig(graph=graph, graph_steps=3).validate()
        e = NativeMnistEngine(cfg, x, y, cuda_dev)
        v0 = {k: t.clone() for k, t in e.layout.views(e.params).items()}
        e.train(7)
        torch.cuda.synchronize()
        U = torch.empty_like(e.bufs["wino_u"])
        Ud = torch.empty_like(e.bufs["wino_ud"])
        W = ptr(e.params) + 4 * e.layout.offsets["conv2_weight"]
        Cn.mnist.conv2_wino_weights(W, ptr(U), ptr(Ud), stream_handle())
        torch.cuda.synchronize()
        # same operation order, no FMA contraction: bit-identical transforms
        assert torch.equal(e.bufs["wino_u"], U) and torch.equal(e.bufs["wino_ud"], Ud)
        v1 = e.layout.views(e.params)
        for name in ("conv1_weight", "conv1_bias", "conv2_weight", "conv2_bias"):
            assert not torch.equal(v0[name], v1[name]), f"{name} was not updated"
        assert torch.isfinite(e.params).all()


@pytest.mark.parametrize("B", [64, 96, 38])
def test_wino_conv2_bwd_filter_matches_oracle(cuda_dev, B):
    """dW2 / db2 from the Winograd filter-gradient kernel (point slabs) and
    the finalize kernel's G^T M G output transform vs torch autograd in fp64,
    for a pool-scattered dY2 (B = 38: a partial last image group and the
    non-XCD block mapping)."""
    Cn = native()
    g = torch.Generator().manual_seed(13)
    a1 = torch.relu(torch.randn(B, 14, 14, 32, generator=g))
    dpool = torch.randn(B, 7, 7, 64, generator=g)
    q = torch.randint(0, 4, (B, 7, 7, 64), generator=g)
    dy2 = torch.zeros(B, 14, 14, 64)
    for k in range(4):
        dy2[:, k >> 1::2, k & 1::2, :] = torch.where(q == k, dpool, torch.zeros(()))
    a1pf = torch.zeros(B, 18, 18, 32)
    a1pf[:, 2:16, 2:16] = a1
    a1pf, dy2d = a1pf.to(cuda_dev), dy2.to(cuda_dev)
    groups = Cn.mnist.conv2_wino_filter_groups(B)
    part2 = torch.full((Cn.mnist.part2_floats_wino(B),), float("nan"), device=cuda_dev)
    part1 = torch.zeros(832, device=cuda_dev)
    gw2 = torch.empty(5, 5, 32, 64, device=cuda_dev)
    gb2 = torch.empty(64, device=cuda_dev)
    gw1 = torch.empty(800, device=cuda_dev)
    gb1 = torch.empty(32, device=cuda_dev)
    s = stream_handle()
    Cn.mnist.conv2_bwd_filter_wino(ptr(a1pf), ptr(dy2d), B, ptr(part2), s)
    Cn.mnist.grad_finalize(ptr(part2), groups, ptr(part1), 0, ptr(gw2), ptr(gb2), ptr(gw1),
                           ptr(gb1), s)
    torch.cuda.synchronize()
    w = torch.zeros(5, 5, 32, 64, dtype=torch.float64, requires_grad=True)
    z = F.conv2d(a1.permute(0, 3, 1, 2).double(), w.permute(3, 2, 0, 1), padding=2)
    z.backward(dy2.permute(0, 3, 1, 2).double())
    assert torch.isfinite(gw2).all() and torch.isfinite(gb2).all()
    assert _rel(gw2.double().cpu(), w.grad) < 5e-5
    assert _rel(gb2.double().cpu(), dy2.double().sum((0, 1, 2))) < 1e-5
