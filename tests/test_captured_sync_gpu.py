"""Multi-rank checks of the CAPTURED (hipGraph-replayed) training steps with
real cross-rank data on ONE GPU: 2 ranks share the device and exchange their
buckets through the shared-memory communicator (csrc/shm_comm.h), whose
collectives are captured with the step (D2H copy, host-function exchange,
H2D copy).  Every captured sync schedule of the native MNIST executor, the
bf16 gradient wire, the auto-tune (side-effect free) and a captured schedule
switching sequence must be bit-identical to the eager host-staged run and to
the serial emulation; the reference's periodic weight averaging (all-ranks
and the root-only quirk) must equal the mean of the replicas; ResNet-18 and
the fused LeNet-5 executor with captured bucketed sync must equal their
serial emulation.  Reference: the MPI Scatter / Gather data parallelism of
/root/reference/mpipy.py:121-127, :236-241, :87-91."""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HELPER = os.path.join(ROOT, "tests", "helpers", "captured_sync_ranks.py")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(*args, timeout=420):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), HELPER] + list(args)
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    return r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_captured_mnist_schedules_two_ranks(dtype):
    out = _run("mnist", dtype)
    assert f"CAPTURED_SYNC_OK mnist {dtype} world=2" in out, out[-2000:]


@pytest.mark.gpu
def test_param_avg_and_root_only_two_ranks():
    out = _run("param_avg")
    assert "CAPTURED_SYNC_OK param_avg" in out, out[-2000:]


@pytest.mark.gpu
@pytest.mark.parametrize("model", ["resnet18", "lenet5-native"])
def test_captured_generic_bucketed_sync_two_ranks(model):
    out = _run("generic", model)
    assert f"CAPTURED_SYNC_OK generic {model} world=2" in out, out[-2000:]
