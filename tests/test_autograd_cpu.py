"""Autograd checks of the op semantics (SURVEY.md §4 "Unit: autograd"):
torch.autograd.gradcheck in fp64 on the CPU oracle path of every layer op
the models use (NHWC conv / linear / BatchNorm with fused residual + ReLU /
pooling / cross-entropy) and of the reference MNIST model's loss w.r.t. its
parameters.  The GPU kernels are then tested against these oracles
(tests/test_*_gpu.py)."""

import pytest
import torch
from torch.autograd import gradcheck

from mpi_tensorflow_amd.models import mnist_cnn as M
from mpi_tensorflow_amd.ops import functional as Fn

torch.manual_seed(0)
D = torch.float64


def _p(*shape):
    t = (torch.randn(*shape, dtype=D) * 0.3).requires_grad_(True)
    return t


@pytest.mark.parametrize("stride,pad,relu", [(1, 1, False), (2, 1, True), (2, 0, False)])
def test_conv2d_nhwc(stride, pad, relu):
    x, w, b = _p(2, 7, 6, 3), _p(3, 3, 3, 4), _p(4)

    def f(x, w, b):
        return Fn.conv2d(x, Fn.Param(w, None), Fn.Param(b, None), stride, pad, relu)

    assert gradcheck(f, (x, w, b), eps=1e-6, atol=1e-6)


def test_linear():
    x, w, b = _p(5, 7), _p(7, 3), _p(3)
    assert gradcheck(lambda x, w, b: Fn.linear(x, Fn.Param(w, None), Fn.Param(b, None), True),
                     (x, w, b), eps=1e-6, atol=1e-6)


@pytest.mark.parametrize("relu,res", [(False, False), (True, True)])
def test_batchnorm_training(relu, res):
    x, g, b, r = _p(3, 4, 4, 5), _p(5), _p(5), _p(3, 4, 4, 5)

    def f(x, g, b, r):
        rm, rv = torch.zeros(5, dtype=D), torch.ones(5, dtype=D)
        return Fn.batchnorm(x, Fn.Param(g, None), Fn.Param(b, None), rm, rv, True, relu,
                            r if res else None)

    assert gradcheck(f, (x, g, b, r), eps=1e-6, atol=1e-5)


def test_pooling_and_xent():
    x = _p(2, 6, 6, 3)
    assert gradcheck(lambda x: Fn.maxpool(x, 2, 2), (x,), eps=1e-6, atol=1e-6)
    assert gradcheck(lambda x: Fn.maxpool(x, 3, 2, 1), (x,), eps=1e-6, atol=1e-6)
    assert gradcheck(Fn.global_avgpool, (x,), eps=1e-6, atol=1e-6)
    logits = _p(4, 10)
    labels = torch.tensor([1, 0, 9, 3])
    assert gradcheck(lambda l: Fn.cross_entropy(l, labels), (logits,), eps=1e-6, atol=1e-6)


def test_mnist_cnn_loss_wrt_params():
    """The reference model (mpipy.py:155-167, loss :54-58) with a fixed
    dropout mask: gradients of xent + L2 w.r.t. all 8 parameter tensors."""
    lay = M.layout()
    flat = torch.zeros(lay.total, dtype=torch.float32)
    M.init_params(flat, lay, seed=1)
    views = {k: v.detach().to(D).clone().requires_grad_(True) for k, v in lay.views(flat).items()}
    # fixed inputs: the directional step eps*d moves ~1e-4 of the conv
    # pre-activations, so some draws put ReLU kinks inside the +-eps
    # finite-difference window (a slope change there is an O(1) share of the
    # difference); this draw has none on the checked directions
    torch.manual_seed(2)
    x = torch.rand(2, 28, 28, 1, dtype=D) - 0.5
    y = torch.tensor([3, 7])
    mask = torch.rand(2, M.FC1_OUT) < 0.5
    names = [s.name for s in lay.specs]

    def f(*ps):
        v = dict(zip(names, ps))
        logits = M.forward(v, x, mask, 0.5)
        return torch.nn.functional.cross_entropy(logits, y) + 5e-4 * M.l2_term(v)

    # gradcheck would need 2 forwards per element (1.6 M of them); check every
    # tensor's gradient through random directional derivatives instead
    loss = f(*[views[m] for m in names])
    grads = torch.autograd.grad(loss, [views[m] for m in names])
    gen = torch.Generator().manual_seed(5)
    eps = 1e-6
    for n, gw in zip(names, grads):
        w = views[n]
        for _ in range(2):
            d = torch.randn(w.shape, generator=gen, dtype=D)
            with torch.no_grad():
                lp = f(*[(w + eps * d) if m == n else views[m] for m in names])
                lm = f(*[(w - eps * d) if m == n else views[m] for m in names])
            fd = ((lp - lm) / (2 * eps)).item()
            an = (gw * d).sum().item()
            assert abs(fd - an) < 1e-6 * max(1.0, abs(fd)), (n, fd, an)
