"""Failure detection, launcher and checkpoint robustness (CPU).

* the collective watchdog (parallel/watchdog.py) turns a hung region or an
  RCCL asynchronous error into an abort of the communicators and a non-zero
  exit (SURVEY §5 failure row; the reference only has MPI's default abort,
  /root/reference/mpipy.py:195-198 being its one, broken, error handler);
* bench.py --gpus N with no launcher starts N ranks itself and rejects a
  world-size mismatch;
* checkpoints: int64 step, BN running statistics, world/model mismatch,
  resume + parameter averaging of a generic (autograd-leaf) model.
"""

import json
import os
import subprocess
import sys
import textwrap
import time

import numpy as np
import pytest
import torch

from test_distributed_cpu import ROOT, _free_port, _run

from mpi_tensorflow_amd.parallel.watchdog import EXIT_CODE, CollectiveWatchdog, make_watchdog


class FakeComm:
    def __init__(self, err_after=None, code=3):
        self.t0 = time.monotonic()
        self.err_after, self.code = err_after, code
        self.aborted = False

    def async_error(self):
        if self.err_after is not None and time.monotonic() - self.t0 > self.err_after:
            return self.code
        return 0

    def abort(self):
        self.aborted = True


def _wait(pred, t=5.0):
    end = time.monotonic() + t
    while time.monotonic() < end:
        if pred():
            return True
        time.sleep(0.01)
    return False


def test_watchdog_deadline_aborts_and_exits():
    codes = []
    c = FakeComm()
    wd = CollectiveWatchdog([c], timeout_s=0.2, rank=3, poll_s=0.01, exit_fn=codes.append)
    wd.arm("train steps 0..24")
    assert _wait(lambda: codes), "watchdog did not fire"
    assert codes == [EXIT_CODE] and c.aborted and "deadline" in wd.fired


def test_watchdog_async_error_fires_even_when_idle():
    codes = []
    c = FakeComm(err_after=0.05, code=6)
    wd = CollectiveWatchdog([c], timeout_s=100.0, poll_s=0.01, exit_fn=codes.append)
    assert _wait(lambda: codes)
    assert c.aborted and "asynchronous error 6" in wd.fired


def test_watchdog_guard_disarms_and_in_progress_is_not_an_error():
    codes = []
    c = FakeComm(err_after=0.0, code=7)  # ncclInProgress
    wd = CollectiveWatchdog([c], timeout_s=0.1, poll_s=0.01, exit_fn=codes.append)
    with wd.guard("short region"):
        time.sleep(0.02)
    time.sleep(0.3)
    wd.stop()
    assert not codes and not c.aborted


def test_make_watchdog_single_rank_is_noop():
    wd = make_watchdog([FakeComm()], 0.01, 0, 1)
    with wd.guard("x"):
        time.sleep(0.05)
    assert wd.fired is None


def test_watchdog_really_exits_process():
    """A stalled rank (a 'collective' that never completes) exits with
    EXIT_CODE within the deadline instead of hanging."""
    code = textwrap.dedent(f"""
        import sys, time
        sys.path.insert(0, {ROOT!r})
        from mpi_tensorflow_amd.parallel.watchdog import CollectiveWatchdog
        class Stuck:
            def async_error(self): return 0
            def abort(self): print("aborted", flush=True)
        wd = CollectiveWatchdog([Stuck()], timeout_s=1.0, rank=1)
        with wd.guard("all-reduce of bucket 1"):
            time.sleep(60)   # the device synchronize that never returns
        print("unreachable")
    """)
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    dt = time.monotonic() - t0
    assert r.returncode == EXIT_CODE, (r.stdout, r.stderr)
    assert "aborted" in r.stdout and "unreachable" not in r.stdout
    assert "[rank 1] collective watchdog" in r.stderr and "all-reduce of bucket 1" in r.stderr
    assert dt < 30


@pytest.mark.slow
def test_bench_spawns_ranks_without_launcher():
    out = _run([sys.executable, "bench.py", "--gpus", "2", "--steps", "3", "--warmup", "1",
                "--backend", "torch"])
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    j = json.loads(lines[0])
    assert j["n_gpus"] == 2 and j["config"]["parallelism"] == "dp2"
    assert j["config"]["ranks"] == 2 and j["config"]["global_batch"] == 128
    assert j["config"]["replicas_identical"] is True  # post-run weight checksum over ranks


@pytest.mark.slow
def test_bench_world_mismatch_fails():
    port = _free_port()
    env = dict(os.environ, OMP_NUM_THREADS="2", PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="",
               HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node=2", "--master-addr", "127.0.0.1", "--master-port",
                        str(port), "bench.py", "--gpus", "3", "--steps", "2", "--warmup", "1",
                        "--backend", "torch"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode != 0
    assert "--gpus 3 but the launcher started 2" in r.stderr


# ------------------------------------------------------------- checkpoints
def _generic(model, rows, B, seed=1):
    from mpi_tensorflow_amd import config as C
    from mpi_tensorflow_amd.models.generic import model_input_shape
    from mpi_tensorflow_amd.runtime.generic_engine import GenericEngine
    from mpi_tensorflow_amd.utils.data import synthetic_images_torch

    tx, ty = synthetic_images_torch(rows, model_input_shape(model), seed=seed)
    cfg = C.TrainConfig(model=model, batch_size=B, device="cpu").validate()
    return GenericEngine(cfg, tx.numpy(), ty.numpy(), torch.device("cpu")), tx.numpy(), ty.numpy()


def test_checkpoint_int64_step_and_meta_mismatch(tmp_path):
    from mpi_tensorflow_amd.utils import checkpoint as ck

    eng, x, y = _generic("lenet5", 64, 16)
    eng.train(2)
    p = str(tmp_path / "c.npz")
    big = (1 << 24) + 3  # float32 iter_ cannot hold it
    ck.save(p, eng.layout, eng.params, eng.mom, big, meta={"model": "lenet5", "world": 1})
    e2, _, _ = _generic("lenet5", 64, 16, seed=2)
    step, meta = ck.load(p, e2.layout, e2.params, e2.mom, expect={"model": "lenet5", "world": 1})
    assert step == big and meta["world"] == "1"
    assert torch.equal(e2.params.detach(), eng.params.detach())
    assert torch.equal(e2.mom, eng.mom)
    with pytest.raises(ValueError, match="world"):
        ck.load(p, e2.layout, e2.params, e2.mom, expect={"model": "lenet5", "world": 2})


def test_resnet18_checkpoint_restores_bn_running_stats(tmp_path):
    from mpi_tensorflow_amd.utils import checkpoint as ck

    torch.manual_seed(0)
    eng, x, y = _generic("resnet18", 6, 2)
    eng.train(2)  # moves the running statistics away from (0, 1)
    rm, rv = eng.bn["bn1"]
    assert not torch.allclose(rm, torch.zeros_like(rm))
    err0 = eng.evaluate(x[:4], y[:4])
    with torch.no_grad():
        ref_logits = eng.model.forward(eng.P, eng.bn, torch.from_numpy(x[:4]), False)
    p = str(tmp_path / "r.npz")
    ck.save(p, eng.layout, eng.params, eng.mom, eng.step, meta={"model": "resnet18"},
            extra=eng.extra_state())
    e2, _, _ = _generic("resnet18", 6, 2, seed=5)
    step, _ = ck.load(p, e2.layout, e2.params, e2.mom, extra=e2.extra_state(),
                      expect={"model": "resnet18"})
    e2.set_step(step)
    for k in eng.bn:
        assert torch.equal(eng.bn[k][0], e2.bn[k][0]) and torch.equal(eng.bn[k][1], e2.bn[k][1]), k
    with torch.no_grad():
        got = e2.model.forward(e2.P, e2.bn, torch.from_numpy(x[:4]), False)
    assert torch.equal(got, ref_logits)
    assert e2.evaluate(x[:4], y[:4]) == err0


@pytest.mark.slow
def test_lenet5_resume_then_param_avg_two_ranks(tmp_path):
    """Save, resume, then --sync param_avg at world 2 on the generic engine
    (its params are an autograd leaf: resume and averaging must write its
    storage under no_grad)."""
    ck = str(tmp_path / "l.npz")
    port = _free_port()
    base = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
            "--master-addr", "127.0.0.1", "--master-port"]
    _run(base + [str(port), "mpipy.py", "--device", "cpu", "--model", "lenet5", "--max-steps",
                 "20", "--sync", "param_avg", "--sync-every", "10", "--ckpt", ck, "--quiet"])
    z = np.load(ck, allow_pickle=False)
    assert int(z["__meta__/step"]) == 20 and str(z["__meta__/world"]) == "2"
    out = _run(base + [str(_free_port()), "mpipy.py", "--device", "cpu", "--model", "lenet5",
                       "--max-steps", "41", "--sync", "param_avg", "--sync-every", "10",
                       "--resume", ck, "--check-replicas"])
    summ = json.loads([l for l in out.splitlines() if l.startswith('{"summary"')][-1])["summary"]
    assert summ["world"] == 2 and summ["steps"] == 21


# ------------------------------------------------- heartbeat + start-up faults
def test_run_in_chunks_slow_but_progressing_run_is_not_killed():
    """A run far longer than the deadline, but progressing, is chunked into
    separately armed regions and never declared hung (the old
    trainer armed one deadline around a whole segment)."""
    from mpi_tensorflow_amd.parallel.watchdog import run_in_chunks

    codes = []
    wd = CollectiveWatchdog([FakeComm()], timeout_s=0.4, poll_s=0.01, exit_fn=codes.append)
    sizes = []

    def train(n):
        sizes.append(n)
        time.sleep(0.02 * n)

    t0 = time.monotonic()
    run_in_chunks(wd, train, lambda: None, 90, "train steps", granule=2)
    dt = time.monotonic() - t0
    wd.stop()
    assert dt > 1.5 and not codes and wd.fired is None, (dt, codes, wd.fired)
    assert sum(sizes) == 90 and sizes[0] == 2
    assert all(n % 2 == 0 for n in sizes[:-1]) and max(sizes) * 0.02 < 0.4


def test_run_in_chunks_still_catches_a_hang():
    from mpi_tensorflow_amd.parallel.watchdog import run_in_chunks

    codes = []
    wd = CollectiveWatchdog([FakeComm()], timeout_s=0.3, poll_s=0.01, exit_fn=codes.append)
    state = {"step_s": 0.001}

    def train(n):
        time.sleep(1.0)  # one chunk that never finishes in time

    run_in_chunks(wd, train, lambda: None, 10, "train steps", state=state)
    assert codes == [EXIT_CODE] and "deadline" in wd.fired


def _spawn_ranks(world, args, extra_env):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, OMP_NUM_THREADS="2", PYTHONPATH=ROOT, RANK=str(r),
                   WORLD_SIZE=str(world), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), **extra_env)
        procs.append(subprocess.Popen([sys.executable, "mpipy.py"] + args, cwd=ROOT, env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    return procs


@pytest.mark.parametrize("mode", ["exit", "hang"])
def test_peer_failure_during_startup_ends_every_rank(mode):
    """Rank 1 dies (or hangs) right after the communicator is created, inside
    the start-up region: every rank must exit non-zero within the deadline
    (the watchdog exists before the communicator and guards start-up)."""
    timeout = 8.0
    t0 = time.monotonic()
    procs = _spawn_ranks(2, ["--device", "cpu", "--max-steps", "30", "--eval-every", "0",
                             "--quiet", "--collective-timeout-s", str(timeout)],
                         {"MTA_FAULT": f"1:after_comm:{mode}"})
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=120)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise AssertionError("a rank hung after its peer failed")
        outs.append((p.returncode, out))
    dt = time.monotonic() - t0
    assert all(rc != 0 for rc, _ in outs), outs
    assert "MTA_FAULT" in outs[1][1]
    if mode == "exit":
        assert outs[1][0] == 99
    else:
        assert outs[1][0] == EXIT_CODE and "collective watchdog" in outs[1][1], outs[1]
    assert dt < 60, dt
