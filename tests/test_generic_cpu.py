"""CPU checks of the generic model family (LeNet-5, ResNet-18): parameter
inventory, oracle forward/backward vs torch.nn.functional, CPU training
through the Trainer, and 2-rank gloo DP equivalence."""

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from mpi_tensorflow_amd import config as C
from mpi_tensorflow_amd.models.generic import LeNet5, ResNet18, make_model, model_input_shape
from mpi_tensorflow_amd.ops import functional as Fn


def test_param_counts():
    le = LeNet5()
    assert le.layout.numel == 3 * 25 * 6 + 6 + 6 * 25 * 16 + 16 + 400 * 120 + 120 + 120 * 84 + 84 + 84 * 10 + 10
    rn = ResNet18()
    assert rn.layout.numel == 11_181_642  # torchvision resnet18 with a 10-way head
    assert model_input_shape("resnet18") == (224, 224, 3)
    # buckets are contiguous, in backward (reverse forward) order
    buckets = [s.bucket for s in rn.layout.specs]
    assert buckets == sorted(buckets) and len(set(buckets)) == 6  # ~8 MB buckets of 44.7 MB
    assert {s.bucket for s in le.layout.specs} == {0}  # LeNet-5: one 250 KB bucket
    assert rn.layout.specs[0].name == "fc_b" or rn.layout.specs[0].name == "fc_w"


def test_bucket_plans():
    """parallel/overlap.py plan_layout: every plan tiles the flat buffer with
    contiguous buckets at parameter boundaries in backward order; geo:4 puts
    ResNet-18's layer4 (+ head), layer3 and the rest in three buckets."""
    from mpi_tensorflow_amd.parallel.overlap import BUCKET_PLANS, check_plan, plan_layout

    L = ResNet18().layout
    for plan in BUCKET_PLANS + ("bytes:8", "geo:2"):
        check_plan(plan)
        pl = plan_layout(L, plan)
        b = pl.buckets()  # raises unless contiguous and covering
        ids = [s.bucket for s in pl.specs]
        assert ids == sorted(ids) and set(ids) == set(range(len(b)))
        assert [s.name for s in pl.specs] == [s.name for s in L.specs]
    assert plan_layout(L, "layout").buckets() == L.buckets()
    assert len(plan_layout(L, "one").buckets()) == 1
    geo = plan_layout(L, "geo:4")
    first = {s.name.split("_")[0] for s in geo.specs if s.bucket == 0}
    assert [round(4 * (hi - lo) / 1e6, 1) for lo, hi in geo.buckets()] == [33.6, 8.4, 2.7]
    assert all(n.startswith(("fc", "l4")) for n in first), first
    for bad in ("geo:1", "bytes:0", "two", "geo:x"):
        with pytest.raises(ValueError):
            check_plan(bad)
    with pytest.raises(ValueError):
        C.TrainConfig(bucket_plan="geo:1").validate()


def _nchw_lenet(flat_views, x):
    v = flat_views
    h = F.conv2d(x.permute(0, 3, 1, 2), v["c1_w"].permute(3, 2, 0, 1), v["c1_b"]).relu()
    h = F.max_pool2d(h, 2)
    h = F.conv2d(h, v["c2_w"].permute(3, 2, 0, 1), v["c2_b"]).relu()
    h = F.max_pool2d(h, 2).permute(0, 2, 3, 1).reshape(x.shape[0], 400)
    h = (h @ v["f1_w"] + v["f1_b"]).relu()
    h = (h @ v["f2_w"] + v["f2_b"]).relu()
    return h @ v["f3_w"] + v["f3_b"]


def test_lenet_forward_matches_nchw_reference():
    m = LeNet5()
    flat = torch.zeros(m.layout.total)
    m.init_params(flat, 3)
    P = {k: Fn.Param(v, None) for k, v in m.layout.views(flat).items()}
    x = torch.randn(5, 32, 32, 3, generator=torch.Generator().manual_seed(0))
    out = m.forward(P, {}, x, True)
    ref = _nchw_lenet(m.layout.views(flat), x)
    assert out.shape == (5, 10)
    assert torch.allclose(out, ref, atol=1e-5, rtol=1e-5)


def test_resnet_cpu_step_matches_autograd_of_torch_bn():
    """One oracle step at a small spatial size: finite loss and grads, the
    flat momentum-SGD update, and BN running statistics updated."""
    from mpi_tensorflow_amd.runtime.generic_engine import GenericEngine
    from mpi_tensorflow_amd.utils.data import synthetic_rows

    x, y = synthetic_rows("train", 0, 16, shape=(32, 32, 3))
    cfg = C.TrainConfig(model="resnet18", batch_size=4, device="cpu").validate()
    eng = GenericEngine(cfg, x, y, torch.device("cpu"))
    p0 = eng.params.detach().clone()
    eng._step_cpu()
    assert np.isfinite(eng.loss_value())
    assert eng.loss_value() > 0
    g = eng.grads
    assert torch.isfinite(g).all() and g.abs().sum() > 0
    # momentum SGD from zero momentum: p1 = p0 - lr * g
    assert torch.allclose(eng.params.detach(), p0 - eng.lr(0) * g, atol=1e-7)
    # BN running stats moved
    rm, rv = eng.bn["bn1"]
    assert rm.abs().sum() > 0


@pytest.mark.parametrize("model", ["lenet5"])
def test_trainer_generic_cpu(model, tmp_path):
    from mpi_tensorflow_amd.runtime.trainer import Trainer

    cfg = C.TrainConfig(model=model, device="cpu", max_steps=30, eval_every=0, quiet=True,
                        ckpt=str(tmp_path / "ck.npz")).validate()
    tr = Trainer(cfg)
    s = tr.run()
    assert s.steps == 30 and s.model == model
    assert np.isfinite(s.final_loss)
    assert 0.0 <= s.final_test_error_global <= 100.0
    assert (tmp_path / "ck.npz").exists()


def test_lenet_learns_on_cpu():
    from mpi_tensorflow_amd.runtime.generic_engine import GenericEngine
    from mpi_tensorflow_amd.utils.data import synthetic_rows

    x, y = synthetic_rows("train", 0, 2048, shape=(32, 32, 3))
    tx, ty = synthetic_rows("test", 0, 512, shape=(32, 32, 3))
    eng = GenericEngine(C.TrainConfig(model="lenet5", device="cpu").validate(), x, y,
                        torch.device("cpu"))
    e0 = eng.evaluate(tx, ty)
    eng.train(200)
    e1 = eng.evaluate(tx, ty)
    assert e1 < e0 and e1 < 50.0, (e0, e1)


def _worker_lenet_dp(rank, world, port, out_dir, steps):
    import os

    torch.set_num_threads(2)
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from mpi_tensorflow_amd.parallel import dist as D
    from mpi_tensorflow_amd.parallel.comm import make_comm
    from mpi_tensorflow_amd.runtime.generic_engine import GenericEngine
    from mpi_tensorflow_amd.utils.data import synthetic_rows

    di = D.init("cpu")
    comm = make_comm(di, torch.device("cpu"))
    x, y = synthetic_rows("train", rank * 256, (rank + 1) * 256, shape=(32, 32, 3))
    eng = GenericEngine(C.TrainConfig(model="lenet5", device="cpu").validate(), x, y,
                        torch.device("cpu"), rank, world, comm)
    eng.train(steps)
    np.save(os.path.join(out_dir, f"p{rank}.npy"), eng.params.detach().numpy())
    D.shutdown()


@pytest.mark.slow
def test_lenet_dp_gloo_matches_serial(tmp_path):
    """2-rank gloo DP == serial emulation with averaged per-rank grads."""
    import socket

    import torch.multiprocessing as mp

    from mpi_tensorflow_amd.runtime.generic_engine import GenericEngine
    from mpi_tensorflow_amd.utils.data import synthetic_rows

    sck = socket.socket()
    sck.bind(("127.0.0.1", 0))
    port = sck.getsockname()[1]
    sck.close()
    world, steps = 2, 3
    mp.spawn(_worker_lenet_dp, args=(world, port, str(tmp_path), steps), nprocs=world, join=True)
    p0, p1 = np.load(tmp_path / "p0.npy"), np.load(tmp_path / "p1.npy")
    assert np.array_equal(p0, p1)
    cfg = C.TrainConfig(model="lenet5", device="cpu").validate()
    engs = []
    for r in range(world):
        x, y = synthetic_rows("train", r * 256, (r + 1) * 256, shape=(32, 32, 3))
        engs.append(GenericEngine(cfg, x, y, torch.device("cpu"), r, world, None))
    lead = engs[0]
    for s in range(steps):
        gsum = torch.zeros_like(lead.grads)
        for e in engs:
            with torch.no_grad():
                e.params.copy_(lead.params)
                e.mom.copy_(lead.mom)
            e.step = s
            e.params.grad = None
            from mpi_tensorflow_amd.utils.data import batch_offset
            off = batch_offset(s, e.n_local, e.B)
            logits = e.model.forward(e.P, e.bn, e.train_x[off:off + e.B], True)
            Fn.cross_entropy(logits, e.train_y[off:off + e.B]).backward()
            gsum += e.params.grad
        with torch.no_grad():
            lead.mom.mul_(cfg.momentum).add_(gsum / world)
            lead.params.sub_(lead.lr(s) * lead.mom)
    assert np.allclose(p0, lead.params.detach().numpy(), atol=2e-6)


def test_make_model_unknown():
    with pytest.raises(KeyError):
        make_model("vgg")


@pytest.mark.parametrize("model", ["mnist_cnn", "lenet5"])
def test_prediction_heads_cpu(model):
    """train_prediction / eval_prediction (reference mpipy.py:67-68): softmax
    probabilities whose argmax reproduces evaluate()'s error."""
    from mpi_tensorflow_amd.runtime.trainer import Trainer

    cfg = C.TrainConfig(model=model, device="cpu", max_steps=5, eval_every=0, quiet=True,
                        synthetic=True).validate()
    tr = Trainer(cfg)
    tr.run()
    x, y = tr.shard.test_x[:200], tr.shard.test_y[:200]
    p = tr.eval_prediction(x, dropout=False)
    assert p.shape == (200, 10)
    assert torch.allclose(p.sum(1), torch.ones(200, dtype=p.dtype), atol=1e-5)
    err = 100.0 * float((p.argmax(1).cpu().numpy() != y).sum()) / 200
    assert abs(err - tr.engine.evaluate(x, y, dropout=False)) < 1e-9
    tp = tr.train_prediction()
    assert tp.shape == (cfg.batch_size, 10) and torch.isfinite(tp).all()
