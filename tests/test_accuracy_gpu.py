"""Full-run accuracy: the native fp32 and bf16 MNIST engines must reach the
fp32 PyTorch oracle's final test error over the reference's complete run
(2 local epochs at batch 64 = 1562 steps on one rank, mpipy.py:18, :79) on
the v2 synthetic task, which is NOT trivially separable (the oracle ends near
90 %, utils/data.py), so a numerically wrong kernel that still "learns"
shows up as an accuracy gap.  All three runs share the data, the init and the
dropout stream; they differ only in rounding, so the tolerance covers the
trajectory drift that rounding alone causes (docs/ACCURACY.md)."""

import os

import pytest
import torch

from mpi_tensorflow_amd import config as C
from mpi_tensorflow_amd.runtime.mnist_engine import NativeMnistEngine, TorchMnistEngine
from mpi_tensorflow_amd.utils.data import load_mnist_shard, steps_per_run

pytestmark = pytest.mark.gpu
TOL_POINTS = 0.8


@pytest.fixture(scope="module")
def shard():
    return load_mnist_shard(0, 1, synthetic=True)


@pytest.fixture(scope="module")
def oracle_err(cuda_dev, shard):
    cfg = C.TrainConfig(graph=False).validate()
    eng = TorchMnistEngine(cfg, shard.train_x, shard.train_y, cuda_dev)
    eng.train(steps_per_run(eng.n_local, cfg.epochs, cfg.batch_size))
    err = eng.evaluate(shard.test_x, shard.test_y)
    print(f"oracle fp32: final test error {err:.2f}% after {eng.step} steps")
    assert 2.0 < err < 20.0, "synthetic task too easy / too hard to carry information"
    return err


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_native_full_run_matches_oracle_accuracy(cuda_dev, shard, oracle_err, dtype):
    cfg = C.TrainConfig(dtype=dtype, graph=True, graph_steps=25).validate()
    eng = NativeMnistEngine(cfg, shard.train_x, shard.train_y, cuda_dev)
    steps = steps_per_run(eng.n_local, cfg.epochs, cfg.batch_size)
    eng.train(steps)
    torch.cuda.synchronize()
    err = eng.evaluate(shard.test_x, shard.test_y)
    print(f"native {dtype}: final test error {err:.2f}% (oracle {oracle_err:.2f}%) after {steps} steps")
    assert abs(err - oracle_err) <= TOL_POINTS


# ---------------------------------------------------------------- LeNet-5
LENET_TOL_POINTS = 1.0


def test_lenet5_native_full_run_matches_oracle_accuracy(cuda_dev):
    """LeNet-5 (BASELINE config 4) on the v2 CIFAR-shaped task: the native
    fused executor's full run (2 epochs of the 8192-row shard, 256 steps at
    B = 64) must end within 1 point of the fp32 PyTorch oracle's (generic
    engine on the CPU, same data and init).  The oracle must land in 70-95 %,
    i.e. the task is not separable at a glance."""
    from mpi_tensorflow_amd.runtime.generic_engine import GenericEngine
    from mpi_tensorflow_amd.runtime.lenet_engine import NativeLenetEngine
    from mpi_tensorflow_amd.utils.data import synthetic_image_shard

    sh = synthetic_image_shard(0, 1, 8192, 2048, (32, 32, 3))
    cfg = C.TrainConfig(model="lenet5", batch_size=64, graph_steps=16).validate()
    steps = steps_per_run(sh.train_x.shape[0], cfg.epochs, cfg.batch_size)
    ref = GenericEngine(C.TrainConfig(model="lenet5", batch_size=64, device="cpu").validate(),
                        sh.train_x, sh.train_y, torch.device("cpu"))
    ref.train(steps)
    acc_ref = 100.0 - ref.evaluate(sh.test_x, sh.test_y)
    nat = NativeLenetEngine(cfg, sh.train_x, sh.train_y, cuda_dev)
    nat.train(steps)
    torch.cuda.synchronize()
    acc = 100.0 - nat.evaluate(sh.test_x, sh.test_y)
    print(f"lenet5: native {acc:.2f}% vs CPU oracle {acc_ref:.2f}% after {steps} steps")
    assert 70.0 < acc_ref < 95.0, "LeNet-5 task too easy / too hard to carry information"
    assert abs(acc - acc_ref) <= LENET_TOL_POINTS


# -------------------------------------------------------------- ResNet-18
RESNET_STEPS = 200
# max |mean loss| gap per 25-step window, fp32 vs bf16.  Each window averages 5
# single-batch (B = 16) losses, so a changed summation order in either engine
# moves it: measured 0.113 and 0.133 on two builds of round 3 (the fp32 tile
# plans changed in between), against a first-window loss of ~2.2
RESNET_CURVE_TOL = 0.2


def test_resnet18_bf16_tracks_fp32_loss_curve(cuda_dev):
    """ResNet-18 (BASELINE config 5) on the v2 224x224x3 task: the native bf16
    MFMA engine's loss curve over 200 steps must track the native fp32
    engine's (same data, init and batch order) within RESNET_CURVE_TOL per
    25-step window, both must learn, and the held-out accuracy must be
    informative (below 100 %)."""
    from mpi_tensorflow_amd.runtime.generic_engine import GenericEngine
    from mpi_tensorflow_amd.utils.data import synthetic_images_torch

    tx, ty = synthetic_images_torch(1024, (224, 224, 3), device=cuda_dev)
    ex, ey = synthetic_images_torch(256, (224, 224, 3), device=cuda_dev, split="test")
    tx, ty, ex, ey = tx.cpu().numpy(), ty.numpy(), ex.cpu().numpy(), ey.numpy()
    curves, accs = {}, {}
    for dt in ("fp32", "bf16"):
        cfg = C.TrainConfig(model="resnet18", batch_size=16, dtype=dt, graph_steps=25).validate()
        e = GenericEngine(cfg, tx, ty, cuda_dev)
        windows = []
        for _ in range(RESNET_STEPS // 25):
            losses = []
            for _ in range(5):
                e.train(5)
                losses.append(e.loss_value())
            windows.append(sum(losses) / len(losses))
        curves[dt] = windows
        accs[dt] = 100.0 - e.evaluate(ex, ey)
    gap = max(abs(a - b) for a, b in zip(curves["fp32"], curves["bf16"]))
    print(f"resnet18: fp32 curve {[round(v, 3) for v in curves['fp32']]}, bf16 curve "
          f"{[round(v, 3) for v in curves['bf16']]}, max window gap {gap:.3f}; acc fp32 "
          f"{accs['fp32']:.1f}% bf16 {accs['bf16']:.1f}%")
    assert curves["fp32"][-1] < 0.8 * curves["fp32"][0], "fp32 did not learn"
    assert gap <= RESNET_CURVE_TOL
    assert accs["fp32"] < 100.0 and accs["bf16"] < 100.0


# ------------------------------------------- ResNet-18 vs a PyTorch oracle
RESNET_ORACLE_STEPS = 1500
RESNET_ORACLE_ROWS, RESNET_ORACLE_TEST = 4096, 1024
# held-out accuracy gap to the oracle, points (at 1,500 steps,
# where the oracle itself has settled)
RESNET_ORACLE_TOL = {"fp32": 1.0, "bf16": 1.5}


@pytest.fixture(scope="module")
def resnet_task(cuda_dev):
    from mpi_tensorflow_amd.utils.data import synthetic_images_torch

    tx, ty = synthetic_images_torch(RESNET_ORACLE_ROWS, (224, 224, 3), device=cuda_dev)
    ex, ey = synthetic_images_torch(RESNET_ORACLE_TEST, (224, 224, 3), device=cuda_dev,
                                    split="test")
    return tx.cpu().numpy(), ty.numpy(), ex.cpu().numpy(), ey.numpy()


def _resnet_run(cuda_dev, task, dtype, oracle=False):
    from mpi_tensorflow_amd.runtime.generic_engine import GenericEngine

    tx, ty, ex, ey = task
    cfg = C.TrainConfig(model="resnet18", batch_size=32, dtype=dtype, graph=not oracle,
                        graph_steps=25).validate()
    e = GenericEngine(cfg, tx, ty, cuda_dev, oracle=oracle)
    e.train(RESNET_ORACLE_STEPS)
    torch.cuda.synchronize()
    acc = 100.0 - e.evaluate(ex, ey)
    loss = e.loss_value()
    del e
    torch.cuda.empty_cache()
    return acc, loss


# The oracle's (GenericEngine(oracle=True): F.conv2d / F.batch_norm autograd in
# fp32) held-out accuracy moves with the summation order of its MIOpen
# convolutions, which is not reproducible even between two runs on one box;
# the native engines are deterministic.  The pin therefore compares them with
# the MEAN of recorded oracle runs at RESNET_ORACLE_STEPS (same task, init,
# batch order; scripts/resnet_oracle_lab.py --steps 1000,1500):
#   round 4 (closing build, one box):        91.02, 90.82 %
#   round 5 (scripts/sessions/r5_s5.steps, one box):  90.43, 90.33 %
# spread 0.69 points, mean 90.65 %.  MTA_LIVE_ORACLE=1 also runs the oracle
# live (test_resnet18_live_oracle_within_recorded_spread, ~1 min).
RESNET_ORACLE_RUNS = (91.02, 90.82, 90.43, 90.33)


@pytest.fixture(scope="module")
def resnet_oracle_acc():
    return sum(RESNET_ORACLE_RUNS) / len(RESNET_ORACLE_RUNS)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_resnet18_native_matches_torch_oracle_accuracy(cuda_dev, resnet_task, resnet_oracle_acc,
                                                       dtype):
    """ResNet-18 (BASELINE config 5): the native engine (fp32 tiled MFMA or
    bf16 MFMA convs, fused BatchNorm statistics, hipGraph replay) trained
    RESNET_ORACLE_STEPS steps at B = 32 on the v2 224x224x3 task lands within
    RESNET_ORACLE_TOL points of held-out accuracy of a PyTorch-op oracle of
    the same model (same init, data and batch order; the mean of its measured
    runs, RESNET_ORACLE_RUNS)."""
    acc, loss = _resnet_run(cuda_dev, resnet_task, dtype)
    print(f"resnet18 native {dtype}: held-out {acc:.2f}% (oracle {resnet_oracle_acc:.2f}%), "
          f"last loss {loss:.3f}")
    assert abs(acc - resnet_oracle_acc) <= RESNET_ORACLE_TOL[dtype]


@pytest.mark.skipif(os.environ.get("MTA_LIVE_ORACLE") != "1",
                    reason="opt-in (MTA_LIVE_ORACLE=1): a live ResNet-18 oracle run")
def test_resnet18_live_oracle_within_recorded_spread(cuda_dev, resnet_task, resnet_oracle_acc):
    """A live run of the PyTorch-op oracle lands within 0.5 points of the
    recorded runs' range (its data, init and batch-order plumbing - shared
    with the native engines - still produce the recorded task)."""
    acc, _ = _resnet_run(cuda_dev, resnet_task, "fp32", oracle=True)
    lo, hi = min(RESNET_ORACLE_RUNS), max(RESNET_ORACLE_RUNS)
    print(f"resnet18 oracle live: {acc:.2f}% (recorded {lo:.2f}-{hi:.2f}%)")
    assert lo - 0.5 <= acc <= hi + 0.5
