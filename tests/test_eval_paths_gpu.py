"""Evaluation / prediction paths of the GPU engines: the
device copy of an evaluation set is reused only for the same host array
object, labels are never cached, so
  * eval_prediction(test_x) followed by evaluate() scores against the real
    labels (not the placeholder zeros of the prediction call);
  * train_prediction() at different steps returns the rows of different
    batches (temporary slices never hit a stale cache entry);
and the logged loss after graph replays is the loss of the last step that
actually ran.  Reference heads: /root/reference/mpipy.py:67-68 (softmax of
the training / eval logits), :86 and :169-183 (batched test-set error)."""
import numpy as np
import pytest
import torch

from mpi_tensorflow_amd import config as C


def _trainer(model, B):
    from mpi_tensorflow_amd.runtime.trainer import Trainer

    cfg = C.TrainConfig(model=model, batch_size=B, eval_every=0, quiet=True, graph_steps=2,
                        max_steps=4).validate()
    return Trainer(cfg)


@pytest.mark.gpu
def test_eval_prediction_does_not_poison_evaluate_lenet5():
    tr = _trainer("lenet5", 64)
    tr.engine.train(20)
    err0 = tr.evaluate()
    probs = tr.eval_prediction(tr.shard.test_x)  # same object, placeholder labels
    assert probs.shape == (tr.shard.test_x.shape[0], 10)
    err1 = tr.evaluate()
    assert err1 == err0, (err0, err1)
    pred = probs.argmax(1).cpu().numpy()
    want = 100.0 * float((pred != tr.shard.test_y).mean())
    assert abs(want - err0) < 1e-9, (want, err0)


@pytest.mark.gpu
def test_train_prediction_follows_the_step_lenet5():
    tr = _trainer("lenet5", 64)
    a = tr.train_prediction()
    tr.engine.train(1)  # next batch offset
    b = tr.train_prediction()
    assert a.shape == b.shape == (64, 10)
    assert not torch.equal(a, b), "train_prediction returned the previous batch"
    # a slice at the same offset as a fresh array object gives the same rows
    off = tr.engine.step * 64 % (tr.shard.train_x.shape[0] - 64)
    c = tr.eval_prediction(np.array(tr.shard.train_x[off:off + 64]), dropout=True)
    assert torch.equal(b, c)


@pytest.mark.gpu
def test_generic_engine_eval_cache_and_graph_loss_resnet18():
    from mpi_tensorflow_amd.models.generic import model_input_shape
    from mpi_tensorflow_amd.runtime.generic_engine import GenericEngine
    from mpi_tensorflow_amd.utils.data import synthetic_images_torch

    dev = torch.device("cuda")
    x, y = synthetic_images_torch(32, model_input_shape("resnet18"), seed=1)
    x, y = x.numpy(), y.numpy()
    mk = lambda graph: GenericEngine(C.TrainConfig(model="resnet18", batch_size=4, graph=graph,  # noqa: E731
                                                   graph_steps=2).validate(), x, y, dev)
    g, e = mk(True), mk(False)
    g.capture(5)  # 3 eager warm-up steps + the 2-step and the 1-step graphs
    g.train(4)  # replays only the 2-step graph
    e.train(7)
    torch.cuda.synchronize()
    assert torch.equal(g.params.detach(), e.params.detach())
    assert g.loss_value() == e.loss_value(), (g.loss_value(), e.loss_value())
    xs = x[:8]
    err_a, la = g.evaluate(xs, np.zeros(8, np.int64), return_logits=True)
    err_b, lb = g.evaluate(xs, y[:8], return_logits=True)
    assert torch.equal(la, lb)
    want = 100.0 * float((lb.argmax(1).cpu().numpy() != y[:8]).mean())
    assert err_b == want and err_a == 100.0 * float((lb.argmax(1).cpu().numpy() != 0).mean())
    _, l2 = g.evaluate(x[8:16], y[8:16], return_logits=True)  # a different temporary slice
    assert not torch.equal(l2, lb)
