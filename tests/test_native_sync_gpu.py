"""Multi-rank check of the native executor's gradient-sync schedules on ONE
GPU: 2 ranks share the device and talk through a host-staged gloo
communicator (parallel/comm.py:HostStagedComm), so the bucketed all-reduce
and the sharded FC update (reduce-scatter -> 1/N-shard SGD -> all-gather,
csrc/mnist_executor.cpp:train_step_sharded) run with real cross-rank data.
Replaces the reference's MPI weight sync (/root/reference/mpipy.py:95-153)
check "replicas agree" with a bit-exact schedule-equivalence test."""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_sharded_schedule_matches_buckets_two_ranks(dtype):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "helpers", "native_sync_ranks.py"), "6", dtype]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert f"NATIVE_SYNC_OK world=2 steps=6 dtype={dtype}" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("model,steps,batch,wire", [("lenet5", 5, 64, "fp32"),
                                                    ("resnet18", 3, 4, "fp32"),
                                                    ("lenet5-native", 6, 64, "fp32"),
                                                    ("lenet5", 5, 64, "bf16"),
                                                    ("lenet5-native", 6, 64, "bf16")])
def test_generic_bucketed_allreduce_matches_serial_two_ranks(model, steps, batch, wire):
    """Backward-overlapped bucketed all-reduce (parallel/overlap.py) with real
    cross-rank sums vs a serial averaged-gradient emulation: bit-identical."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "helpers", "generic_sync_ranks.py"), model, str(steps),
           str(batch), wire]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert f"GENERIC_SYNC_OK model={model} world=2" in r.stdout and f"wire={wire}" in r.stdout
