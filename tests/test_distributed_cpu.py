"""Multi-rank data parallelism without a cluster: gloo on CPU, world size 2.

Covers the DP sync strategies of parallel/sync.py and the engines'
per-step gradient all-reduce (reference mpipy.py:87-91, :95-153 replaced by
all-reduce semantics), plus the launcher paths (torchrun for mpipy.py and
bench.py)."""

import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(rank, world, port):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    for k in ("OMPI_COMM_WORLD_RANK", "PMI_RANK", "SLURM_PROCID"):
        os.environ.pop(k, None)


def _worker_grad_sync(rank, world, port, out_dir, steps, wire="fp32"):
    torch.set_num_threads(2)
    _env(rank, world, port)
    from mpi_tensorflow_amd import config as C
    from mpi_tensorflow_amd.parallel import dist as D
    from mpi_tensorflow_amd.parallel.comm import make_comm
    from mpi_tensorflow_amd.runtime.mnist_engine import TorchMnistEngine
    from mpi_tensorflow_amd.utils.data import synthetic_rows

    di = D.init("cpu")
    comm = make_comm(di, torch.device("cpu"))
    x, y = synthetic_rows("train", rank * 512, (rank + 1) * 512)
    cfg = C.TrainConfig(device="cpu", grad_comm_dtype=wire).validate()
    eng = TorchMnistEngine(cfg, x, y, torch.device("cpu"), rank, world, comm)
    eng.train(steps)
    np.save(os.path.join(out_dir, f"p{rank}.npy"), eng.params.numpy())
    D.shutdown()


@pytest.mark.slow
@pytest.mark.parametrize("wire", ["fp32", "bf16"])
def test_grad_allreduce_keeps_replicas_identical_and_matches_serial(tmp_path, wire):
    """Per-step gradient all-reduce over gloo (fp32, or the bf16 gradient wire
    of --grad-comm-dtype: every rank's grads and their sum rounded to bf16)
    vs a serial emulation."""
    world, steps, port = 2, 3, _free_port()
    mp.spawn(_worker_grad_sync, args=(world, port, str(tmp_path), steps, wire), nprocs=world,
             join=True)
    p0 = np.load(tmp_path / "p0.npy")
    p1 = np.load(tmp_path / "p1.npy")
    assert np.array_equal(p0, p1), "replicas diverged under per-step gradient all-reduce"

    # serial emulation: average the two ranks' gradients each step
    from mpi_tensorflow_amd import config as C
    from mpi_tensorflow_amd.runtime.mnist_engine import TorchMnistEngine
    from mpi_tensorflow_amd.utils.data import synthetic_rows

    cfg = C.TrainConfig(device="cpu").validate()
    engs = []
    for r in range(world):
        x, y = synthetic_rows("train", r * 512, (r + 1) * 512)
        engs.append(TorchMnistEngine(cfg, x, y, torch.device("cpu"), r, world, None))
    lead = engs[0]
    _, l2_end = lead.layout.l2_range()
    rnd = (lambda t: t.to(torch.bfloat16).float()) if wire == "bf16" else (lambda t: t)
    for s in range(steps):
        gsum = torch.zeros_like(lead.grads)
        for e in engs:
            e.params.copy_(lead.params)
            e.forward_backward(s)
            gsum += rnd(e.grads)
        g = rnd(gsum) / world
        g[:l2_end] += cfg.l2 * lead.params[:l2_end]
        lead.mom.mul_(cfg.momentum).add_(g)
        lead.params.sub_(lead.lr(s) * lead.mom)
    np.testing.assert_allclose(p0, lead.params.numpy(), rtol=0, atol=1e-5)


def _worker_param_avg(rank, world, port, out_dir, quirks):
    torch.set_num_threads(2)
    _env(rank, world, port)
    from mpi_tensorflow_amd import config as C
    from mpi_tensorflow_amd.parallel import dist as D
    from mpi_tensorflow_amd.parallel.comm import make_comm
    from mpi_tensorflow_amd.parallel.sync import average_params, average_params_root_only

    di = D.init("cpu")
    comm = make_comm(di, torch.device("cpu"))
    from mpi_tensorflow_amd.models import mnist_cnn as M

    lay = M.layout()
    p = torch.full((lay.total,), float(rank + 1))
    before = p.clone()
    if quirks:
        average_params_root_only(comm, lay, p)
    else:
        average_params(comm, p)
    np.save(os.path.join(out_dir, f"a{rank}.npy"), p.numpy())
    np.save(os.path.join(out_dir, f"b{rank}.npy"), before.numpy())
    D.shutdown()


@pytest.mark.parametrize("quirks", [False, True])
def test_param_averaging(tmp_path, quirks):
    world, port = 2, _free_port()
    mp.spawn(_worker_param_avg, args=(world, port, str(tmp_path), quirks), nprocs=world, join=True)
    from mpi_tensorflow_amd.models import mnist_cnn as M

    lay = M.layout()
    a0, a1 = np.load(tmp_path / "a0.npy"), np.load(tmp_path / "a1.npy")
    if not quirks:  # all ranks receive the mean of everything
        assert np.allclose(a0, 1.5) and np.allclose(a1, 1.5)
    else:  # Q11: rank 0 averages the four WEIGHT tensors only; rank 1 untouched
        assert np.allclose(a1, 2.0)
        for s in lay.specs:
            lo, hi = lay.segment(s.name)
            want = 1.5 if s.name.endswith("weight") else 1.0
            assert np.allclose(a0[lo:hi], want), s.name


def _run(cmd, timeout=600):
    env = dict(os.environ, OMP_NUM_THREADS="2", PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="",
               HIP_VISIBLE_DEVICES="")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    return r.stdout


@pytest.mark.slow
def test_mpipy_torchrun_two_ranks_param_avg(tmp_path):
    port = _free_port()
    out = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                "--master-addr", "127.0.0.1", "--master-port", str(port), "mpipy.py", "--device",
                "cpu", "--max-steps", "101", "--sync", "param_avg", "--metrics-jsonl",
                str(tmp_path / "m.jsonl"), "--ckpt", str(tmp_path / "ck.npz")])
    assert "Process ID: 0  training session starts!" in out
    assert "Process ID: 1  training session starts!" in out
    assert "0  process at  50 with test error:" in out and "1  process at  100 with test error:" in out
    summ = json.loads([l for l in out.splitlines() if l.startswith('{"summary"')][-1])["summary"]
    assert summ["world"] == 2 and summ["steps"] == 101 and summ["comm"] == "torch-gloo"
    recs = [json.loads(l) for l in open(tmp_path / "m.jsonl")]
    assert recs[-1]["final"] and recs[0]["step"] == 50
    assert (tmp_path / "ck.npz").exists()


@pytest.mark.slow
def test_bench_two_ranks_cpu():
    port = _free_port()
    out = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2",
                "--steps", "3", "--warmup", "1", "--backend", "torch"])
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    j = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in j
    assert j["n_gpus"] == 2 and j["steps"] == 3 and j["config"]["global_batch"] == 128
    assert j["config"]["parallelism"] == "dp2" and j["value"] > 0


@pytest.mark.slow
@pytest.mark.parametrize("model", ["mnist_cnn", "lenet5"])
def test_mpipy_torchrun_grad_sync_replicas_identical(tmp_path, model):
    """Per-step gradient all-reduce over gloo: --check-replicas compares the
    ranks' weight checksums at every eval event and at the end (a mismatch
    raises); device_step_ms is reported."""
    port = _free_port()
    out = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                "--master-addr", "127.0.0.1", "--master-port", str(port), "mpipy.py", "--device",
                "cpu", "--model", model, "--max-steps", "41", "--eval-every", "20",
                "--check-replicas", "--collective-timeout-s", "120"])
    summ = json.loads([l for l in out.splitlines() if l.startswith('{"summary"')][-1])["summary"]
    assert summ["world"] == 2 and summ["steps"] == 41 and summ["model"] == model
    assert summ["device_step_ms"] > 0


def _worker_auto_vote(rank, world, port, out_dir, local_world):
    _env(rank, world, port)
    os.environ["LOCAL_WORLD_SIZE"] = str(local_world)
    from unittest import mock

    from mpi_tensorflow_amd.parallel import comm as CM
    from mpi_tensorflow_amd.parallel import dist as D

    di = D.init("cpu")
    # pretend rank 1 sees one GPU while this host runs 2 local ranks; rank 0
    # sees no GPU: the vote must still give every rank the same answer
    ndev = 1 if rank == 1 else 0
    with mock.patch.object(CM.torch.cuda, "device_count", return_value=ndev):
        share, one_host = CM._auto_vote(di)
    with mock.patch.object(CM, "_host_key", return_value=1000 + rank):
        _, split_hosts = CM._auto_vote(di)
    np.save(os.path.join(out_dir, f"v{rank}.npy"), np.array([share, one_host, split_hosts]))
    D.shutdown()


def test_auto_comm_choice_is_a_collective_vote(tmp_path):
    """comm=auto: whether any rank shares its GPU and whether all ranks run
    on one host are decided by a gloo vote, identically on every rank (a
    rank-local decision could send ranks into different communicators'
    set-up collectives and hang them)."""
    port = _free_port()
    mp.spawn(_worker_auto_vote, args=(2, port, str(tmp_path), 2), nprocs=2, join=True)
    v0, v1 = np.load(tmp_path / "v0.npy"), np.load(tmp_path / "v1.npy")
    assert v0.tolist() == v1.tolist() == [True, True, False]
