"""The shared-memory communicator (csrc/shm_comm.h) without a GPU: its
host-only mode runs the same exchange code the captured GPU collectives run
in their host function.  3 processes check every collective (all-reduce,
reduce-scatter, all-gather, broadcast, reduce; fp32 / bf16 / int64; sum /
max) bit for bit against numpy in rank order, that a collective-order
mismatch between ranks fails every rank (race detection) and that a missing
peer turns into a timeout error instead of a hang (failure detection).
The reference's only collectives are blocking mpi4py Scatter / Gather on
host buffers (/root/reference/mpipy.py:121-127, :236-241)."""
import os
import subprocess
import sys
import uuid

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HELPER = os.path.join(ROOT, "tests", "helpers", "shm_comm_ranks.py")


def _run(world, scenario, tmp_path):
    path = str(tmp_path / f"shm-{uuid.uuid4().hex[:8]}")
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    procs = [subprocess.Popen([sys.executable, HELPER, str(r), str(world), path, scenario],
                              cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                              text=True) for r in range(world)]
    outs = []
    for p in procs:
        out, _ = p.communicate(timeout=240)
        outs.append((p.returncode, out))
    return outs


def test_shm_collectives_bit_exact(tmp_path):
    outs = _run(3, "ok", tmp_path)
    for r, (rc, out) in enumerate(outs):
        assert rc == 0, out[-3000:]
        assert f"SHM_OK rank={r} world=3 ops=21" in out, out[-3000:]


def test_shm_collective_order_mismatch_fails_every_rank(tmp_path):
    outs = _run(2, "mismatch", tmp_path)
    for rc, out in outs:
        assert rc == 0 and "SHM_MISMATCH_OK" in out, out[-3000:]


def test_shm_missing_peer_times_out(tmp_path):
    rc, out = _run(2, "timeout", tmp_path)[0]
    assert rc == 0 and "SHM_TIMEOUT_OK rank=0" in out, out[-3000:]


@pytest.mark.parametrize("bad", [dict(nranks=0), dict(rank=2), dict(capacity=0)])
def test_shm_rejects_bad_layout(tmp_path, bad):
    import torch  # noqa: F401
    from mpi_tensorflow_amd.ops import native

    kw = dict(path=str(tmp_path / "x"), create=True, nranks=2, rank=0, capacity=4096,
              timeout_s=1.0, pinned=False)
    kw.update(bad)
    with pytest.raises(RuntimeError):
        native().ShmComm(**kw)


@pytest.mark.parametrize("case", ["multi_host", "shm_fails"])
def test_auto_comm_with_shared_gpus_raises_instead_of_rccl_fallback(monkeypatch, case):
    """comm=auto when ranks share GPUs: with the ranks on several hosts, or
    when the shared-memory set-up fails, no device communicator can work
    (RCCL / a torch `nccl` group rejects two ranks on one device), so
    make_comm raises an error naming the cause instead of returning a
    torch.distributed communicator that would fail later."""
    import torch
    from mpi_tensorflow_amd.parallel import comm as CM
    from mpi_tensorflow_amd.parallel.dist import DistInfo

    di = DistInfo(rank=0, world=2, local_rank=0, local_world=2, launcher="torchrun")
    monkeypatch.setattr(CM, "_auto_vote", lambda _di: (True, case != "multi_host"))

    def no_shm(*a, **k):
        raise RuntimeError("shared-memory communicator unavailable (rank 0: ENOSPC)")

    monkeypatch.setattr(CM, "ShmDeviceComm", no_shm)
    monkeypatch.setattr(CM, "TorchDeviceComm",
                        lambda *a, **k: pytest.fail("fell back to torch.distributed"))
    with pytest.raises(RuntimeError) as ei:
        CM.make_comm(di, torch.device("cuda"), "auto")
    msg = str(ei.value)
    assert ("several hosts" in msg) if case == "multi_host" else ("ENOSPC" in msg and "no fallback" in msg)
