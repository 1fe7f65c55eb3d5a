"""Fused LeNet-5 kernels (csrc/kernels/lenet.hip, runtime/lenet_engine.py)
against the plain-PyTorch fp32 oracle of the same model (models/generic.py
LeNet5 on CPU ops): per-step gradients of every tensor, a multi-step
training trajectory, evaluation, and graph replay == eager launches."""

import numpy as np
import pytest
import torch

from mpi_tensorflow_amd import config as C
from mpi_tensorflow_amd.runtime.generic_engine import GenericEngine
from mpi_tensorflow_amd.runtime.lenet_engine import NativeLenetEngine
from mpi_tensorflow_amd.utils.data import batch_offset, synthetic_rows

pytestmark = pytest.mark.gpu
SHAPE = (32, 32, 3)


@pytest.fixture(scope="module")
def data():
    return synthetic_rows("train", 0, 1024, shape=SHAPE)


def _cfg(**kw):
    return C.TrainConfig(model="lenet5", **kw).validate()


def oracle_grads(params: torch.Tensor, x, y, step, B, n_local):
    """Flat-layout grads of the mean xent on the CPU oracle ops (fp64)."""
    from mpi_tensorflow_amd.models.generic import make_model
    from mpi_tensorflow_amd.ops import functional as Fn

    m = make_model("lenet5")
    lay = m.layout
    p = params.detach().cpu().double().clone().requires_grad_(True)
    g = torch.zeros_like(p)
    pv, gv = lay.views(p), lay.views(g)
    P = {s.name: Fn.Param(pv[s.name], gv[s.name]) for s in lay.specs}
    off = batch_offset(step, n_local, B)
    xb = torch.from_numpy(x[off:off + B]).double()
    yb = torch.from_numpy(np.asarray(y[off:off + B]).astype(np.int64))
    logits = m.forward(P, {}, xb, True)
    loss = torch.nn.functional.cross_entropy(logits, yb)
    (grad,) = torch.autograd.grad(loss, [p])
    return grad.float(), float(loss)


def _nrel(a, b):
    return float((a - b).abs().max() / max(b.abs().max(), 1e-12))


def test_grads_match_oracle(cuda_dev, data):
    x, y = data
    eng = NativeLenetEngine(_cfg(graph=False), x, y, cuda_dev)
    lay = eng.layout
    for step in (0, 3):
        eng.set_step(step)
        eng.forward_backward_only()
        torch.cuda.synchronize()
        ref, ref_loss = oracle_grads(eng.params, x, y, step, eng.B, eng.n_local)
        got = eng.grads.cpu()
        assert abs(eng.loss_rows.mean().item() - ref_loss) < 1e-5 * max(1.0, ref_loss)
        gv, rv = lay.views(got), lay.views(ref)
        errs = {s.name: _nrel(gv[s.name], rv[s.name]) for s in lay.specs}
        print(step, {k: f"{v:.1e}" for k, v in errs.items()})
        for k, e in errs.items():
            assert e < 2e-5, (step, k, e)


def test_training_trajectory_matches_oracle(cuda_dev, data):
    x, y = data
    nat = NativeLenetEngine(_cfg(graph=True, graph_steps=5), x, y, cuda_dev)
    ref = GenericEngine(_cfg(device="cpu"), x, y, torch.device("cpu"))
    ref.params.data.copy_(nat.params.cpu())
    nat.train(12)
    ref.train(12)
    torch.cuda.synchronize()
    d = (nat.params.cpu() - ref.params.detach()).abs().max().item()
    s = ref.params.detach().abs().max().item()
    assert d < 1e-4 * s, d
    assert int(nat.step_dev.item()) == 12 and nat.step == 12
    assert abs(nat.lr_dev.item() - ref.lr(11)) < 1e-9


def test_graph_replay_equals_eager(cuda_dev, data):
    x, y = data
    a = NativeLenetEngine(_cfg(graph=True, graph_steps=4), x, y, cuda_dev)
    b = NativeLenetEngine(_cfg(graph=False), x, y, cuda_dev)
    a.train(10)  # 2 replays of a 4-step graph + a 2-step graph
    b.train(10)
    torch.cuda.synchronize()
    assert torch.equal(a.params, b.params) and torch.equal(a.mom, b.mom)


def test_eval_matches_oracle(cuda_dev, data):
    x, y = data
    tx, ty = synthetic_rows("test", 0, 777, shape=SHAPE)
    nat = NativeLenetEngine(_cfg(), x, y, cuda_dev)
    nat.train(30)
    torch.cuda.synchronize()
    err, logits = nat.evaluate(tx, ty, chunk=300, return_logits=True)
    ref = GenericEngine(_cfg(device="cpu"), x, y, torch.device("cpu"))
    ref.params.data.copy_(nat.params.cpu())
    with torch.no_grad():
        ref_logits = ref.model.forward(ref.P, {}, torch.from_numpy(tx), False)
    assert (logits.cpu() - ref_logits).abs().max().item() < 1e-4 * max(1.0, ref_logits.abs().max().item())
    assert abs(err - ref.evaluate(tx, ty)) < 0.3
