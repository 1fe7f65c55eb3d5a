"""The xGMI peer-to-peer communicator (csrc/xgmi_comm.h, kernels/xgmi.h) and
the MNIST executor's fused sync + SGD schedule (SCHED_XGMI).

The two-rank test maps the OTHER process's buffers through IPC handles and
runs the same kernels, barriers and flag protocol an 8-GPU node runs - only
the peer memory is on the same device here.  Results must be bit-identical to
the eager host-staged buckets schedule and to gloo's sums.  The emulated test
runs the fused launch against 8 virtual ranks on one GPU (stand-in peer
buffers; timing model only) and checks that it trains without a barrier
timeout.  Reference: the reference's weight Gather to rank 0 every 50 steps
(/root/reference/mpipy.py:95-153), replaced by a per-step gradient sync."""
import os
import socket
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HELPER = os.path.join(ROOT, "tests", "helpers", "captured_sync_ranks.py")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_xgmi_two_ranks_bit_identical_to_buckets(dtype):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), HELPER, "xgmi", dtype]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert f"CAPTURED_SYNC_OK xgmi {dtype} world=2" in r.stdout, r.stdout[-2000:]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["xgmi", "xgmipush", "xgmipull"])
def test_xgmi_lenet5_two_ranks_fused_sync_matches_serial(mode):
    """The fused LeNet-5 executor over the xGMI communicator, bit-identical to
    the serial emulation of data parallelism (rank-order sum + flat SGD):
    xgmi - the two-phase launch (this rank's segment summed and updated,
    sharded momentum, then the other segments gathered); xgmipush - the push
    sync in the update launch (every block pushes its gradient values into the
    peers' receive slots, one barrier, rank-order sum, replicated SGD);
    xgmipull - the one-shot launch (every rank's double-buffered gradient slot
    read after one barrier, rank-order sum, replicated SGD, graph-captured
    steps alternating the slots)."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), HELPER, "generic",
           f"lenet5-native-{mode}"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert f"CAPTURED_SYNC_OK generic lenet5-native-{mode} world=2" in r.stdout, r.stdout[-2000:]


@pytest.mark.gpu
def test_xgmi_emulated_eight_ranks_trains(cuda_dev):
    from mpi_tensorflow_amd import config as C
    from mpi_tensorflow_amd.parallel.comm import XgmiDeviceComm
    from mpi_tensorflow_amd.runtime.mnist_engine import NativeMnistEngine
    from mpi_tensorflow_amd.utils.data import synthetic_rows

    x, y = synthetic_rows("train", 0, 1024)
    cfg = C.TrainConfig(graph=True, graph_steps=5).validate()
    comm = XgmiDeviceComm.emulated(8, lat_us=2.0, link_gbps=64.0)
    eng = NativeMnistEngine(cfg, x, y, cuda_dev, 0, 1, comm, force_sync=True)
    assert eng.sync_schedule == "xgmi"
    p0 = eng.params.clone()
    eng.train(10)
    torch.cuda.synchronize()
    assert comm.error() == 0
    assert int(eng.step_dev.item()) == 10
    assert torch.isfinite(eng.params).all() and not torch.equal(eng.params, p0)


@pytest.mark.gpu
def test_xgmi_missing_peer_times_out_and_fails_fast(cuda_dev):
    """Failure detection: a peer that never arrives makes the barrier time out
    (bounded spin), the kernel completes and sets the sticky error bit, and
    every later collective of that communicator skips the wait (fail fast)
    instead of waiting the timeout again - no GPU hang."""
    import time

    from mpi_tensorflow_amd.parallel.comm import XgmiDeviceComm

    comm = XgmiDeviceComm.emulated(4, lat_us=0.0, link_gbps=0.0, timeout_s=0.3)
    comm.native_handle.emulate_dead_rank(2)
    t = torch.ones(1 << 16, device=cuda_dev)
    comm.register(t)
    t0 = time.perf_counter()
    comm.all_reduce_(t)
    torch.cuda.synchronize()
    first = time.perf_counter() - t0
    assert comm.error() == 1
    t0 = time.perf_counter()
    for _ in range(5):
        comm.all_reduce_(t)
    torch.cuda.synchronize()
    later = time.perf_counter() - t0
    print(f"xgmi dead peer: first collective {first * 1e3:.0f} ms, next five {later * 1e3:.1f} ms")
    assert first >= 0.25 and later < 0.25


@pytest.mark.gpu
@pytest.mark.parametrize("n", [2, 3, 8])
def test_xgmi_exactness_gate_emulated_rejects_a_skipped_peer(cuda_dev, n):
    """The gate (parallel/comm.py xgmi_exactness_check): integer data whose
    sum is exact in any order; the all-reduce, reduce-scatter and all-gather
    (64- and 256-thread grids) must match the exact sums bit for bit.  With
    the skip-peer fault (phase-1 sums leave one rank out, which on real ranks
    gives identical replicas with wrong sums) the gate must reject."""
    from mpi_tensorflow_amd.parallel.comm import XgmiDeviceComm, xgmi_exactness_check

    good = XgmiDeviceComm.emulated(n, lat_us=0.0, link_gbps=0.0)
    assert xgmi_exactness_check(good) is None
    bad = XgmiDeviceComm.emulated(n, lat_us=0.0, link_gbps=0.0)
    bad.inject_skip_peer(n - 1)
    why = xgmi_exactness_check(bad)
    assert why is not None and "exact integer sum" in why, why
    assert good.error() == 0 and bad.error() == 0  # wrong sums, no timeout


@pytest.mark.gpu
def test_xgmi_emulated_link_rate_is_not_rounded_away(cuda_dev):
    """the emulated link floor at 150 GB/s was rounded to whole
    ticks a KiB (~102 GB/s); a MiB keeps the rate within 0.1 %."""
    from mpi_tensorflow_amd.parallel.comm import XgmiDeviceComm

    for gbps in (64.0, 150.0, 400.0):
        c = XgmiDeviceComm.emulated(8, 1.0, gbps)
        t = c.native_handle.link_ticks_per_mib
        assert abs((1 << 20) / (t / 1e8) / 1e9 - gbps) / gbps < 2e-3, (gbps, t)


@pytest.mark.gpu
def test_bench_emulated_xgmi_with_skipped_peer_fails_the_gate(cuda_dev):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--xgmi-emulate", "0,0,8",
                        "--xgmi-inject-skip-peer", "5", "--steps", "2", "--warmup", "1",
                        "--no-eval", "--prewarm-ms", "0"],
                       cwd=ROOT, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 5, r.stdout[-2000:] + r.stderr[-3000:]
    assert "exactness check" in r.stderr


@pytest.mark.gpu
def test_xgmi_two_ranks_gate_catches_identical_but_wrong_sums():
    """2 ranks over IPC: the skip-peer fault on both ranks gives bit-identical
    results on the two ranks that are NOT the sum - what a replica checksum
    cannot see.  The exactness gate rejects it, the MNIST auto-tune's trial
    step compare (one xGMI step vs one serial step over the shared-memory
    communicator) rejects every xGMI schedule of a faulty communicator that
    passed the gate before the fault, and accepts them without the fault."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), HELPER, "xgmi_gate"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "CAPTURED_SYNC_OK xgmi_gate" in r.stdout, r.stdout[-2000:]


@pytest.mark.gpu
def test_block_dispatch_order_per_xcd(cuda_dev):
    """The no-deadlock argument of the xGMI per-block barriers (kernels/xgmi.h)
    rests on the dispatcher: no block starts before the lower-id blocks of its
    XCD.  Measured here: block b runs on XCD (b + o) mod 8, o = where the
    dispatcher's round robin stood after the previous launch (first run on the
    box: block 0 on XCD 5), so XCD-aware tilings group ids by b mod 8 and the
    barrier argument uses per-XCD order only.  A grid of 4x the resident
    capacity (64-thread blocks holding their CU 20 us each) records every
    block's XCD and start clock (xgmi.hip dispatch_probe_kernel)."""
    import numpy as np

    from mpi_tensorflow_amd.ops import native, stream_handle

    cus = torch.cuda.get_device_properties(cuda_dev).multi_processor_count
    blocks = cus * 32 * 4
    ctr = torch.zeros(256, dtype=torch.int32, device=cuda_dev)
    out = torch.zeros(3 * blocks, dtype=torch.int64, device=cuda_dev)
    native().mnist.xgmi_dispatch_probe(ctr.data_ptr(), out.data_ptr(), blocks, 2000,
                                       stream_handle())
    torch.cuda.synchronize()
    o = out.cpu().numpy().reshape(blocks, 3)
    xcc, start = o[:, 0], o[:, 2]
    ids = np.arange(blocks)
    nx = len(np.unique(xcc))
    print(f"dispatch probe: {blocks} blocks over {nx} XCDs")
    if nx == 8:
        o = int(xcc[0])
        print(f"dispatch probe: block 0 on XCD {o}")
        assert np.array_equal(xcc, (ids + o) % 8), "blocks are not assigned to XCDs round-robin"
    worst = 0
    for x in np.unique(xcc):
        s = start[xcc == x]  # in id order
        # the latest start among lower ids, against each block's own start
        late = np.maximum.accumulate(s)[:-1] - s[1:]
        worst = max(worst, int(late.max(initial=0)))
    # 2 us of slack for blocks dispatched together on different shader engines
    # (one spin is 20 us: a block dispatched out of order would start >= 20 us
    # before a lower id)
    assert worst <= 200, f"a block started {worst / 100:.1f} us before a lower-id block of its XCD"


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["two-phase", "push", "pull"])
def test_bench_lenet5_emulated_xgmi_modes(cuda_dev, mode):
    """bench.py on 8 emulated xGMI ranks, LeNet-5, each sync mode: one JSON
    line naming the mode, the gate passed, no barrier timed out."""
    import json

    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--model", "lenet5",
                        "--xgmi-emulate", "1,150,8", "--xgmi-mode", mode, "--steps", "50",
                        "--warmup", "10", "--no-eval", "--prewarm-ms", "0"],
                       cwd=ROOT, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    name = {"two-phase": "xgmi", "push": "xgmi-push", "pull": "xgmi-pull"}[mode]
    assert out["config"]["sync_schedule"] == name, out["config"]
    assert out["config"]["xgmi_gate"] == "passed"
    print(f"lenet5 emulated 8 ranks {mode}: {1000 * out['ms_per_step']:.2f} us/step")
