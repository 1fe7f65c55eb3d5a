"""The driver's exact multi-rank entry points, run end to end on ONE GPU.

The round-end scaling bench runs `bench.py --gpus N` (one rank per GPU,
RCCL) and a user of the reference runs `mpirun -np P python mpipy.py`
(/root/reference/README.md:4, mpipy.py:208-241 rank / size / Scatter,
:87-91 + :121-127 the periodic Gather).  These tests run the same scripts
with two ranks that share the one GPU of the test box through the
shared-memory communicator (`--comm shm`, csrc/shm_comm.h): everything
else - spawning, the sync-schedule autotune, hipGraph capture of the synced
step, prewarm, timed replay, the chunked accuracy run, the optimizer-state
gather, the replica fingerprints and the communicator rank check - is the
code path of the N-GPU run.
"""

import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(cmd, timeout=420):
    env = dict(os.environ, PYTHONPATH=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, f"rc={r.returncode}\n{r.stdout[-3000:]}\n{r.stderr[-5000:]}"
    return r.stdout


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


@pytest.mark.parametrize("model,dtype,extra", [
    ("mnist_cnn", "fp32", []),
    ("mnist_cnn", "bf16", []),
    ("lenet5", "fp32", []),
    ("resnet18", "fp32", ["--batch-size", "8", "--no-eval"]),
])
def test_bench_two_ranks_shared_gpu(cuda_dev, model, dtype, extra):
    """`bench.py --gpus 2` spawns its own two ranks (no launcher), exactly as
    the driver's N > 1 runs do apart from the communicator."""
    steps = 10 if model == "resnet18" else 30
    out = _run([sys.executable, "bench.py", "--gpus", "2", "--comm", "shm", "--model", model,
                "--dtype", dtype, "--steps", str(steps), "--warmup", "5"] + extra)
    lines = _json_lines(out)
    assert len(lines) == 1, out
    j = lines[0]
    c = j["config"]
    assert j["n_gpus"] == 2 and j["steps"] == steps and c["parallelism"] == "dp2"
    assert c["comm"] == "host-shm" and c["comm_nranks"] == 2
    assert c["replicas_identical"] is True
    assert c["engine"] in ("native", "native-lenet5", "generic") and j["value"] > 0
    if model == "mnist_cnn":
        assert j["final_test_accuracy"] is not None and j["final_test_accuracy"] > 50.0
    if model == "mnist_cnn" and dtype == "fp32":
        tune = c["sync_tune_us_per_step"]
        assert tune and len([v for v in tune.values() if v is not None]) >= 2, tune
        assert c["sync_schedule"] in tune
    if model == "resnet18":  # the all-reduce bucket plan, tuned at start-up
        tune = c["sync_tune_us_per_step"]
        assert tune and None not in tune.values() and len(set(tune.values())) >= 2, tune
        assert c["sync_schedule"].startswith("buckets(") and c["sync_schedule"][8:-1] in tune
        # every overlapped (non-final) bucket's collective graph moved bytes
        nodes = c["collective_graph_nodes"]
        if c["sync_schedule"] != "buckets(one)":
            assert nodes and all(k > 0 for k in nodes), nodes


@pytest.mark.parametrize("model,dtype", [("mnist_cnn", "fp32"), ("mnist_cnn", "bf16"),
                                         ("lenet5", "fp32")])
def test_bench_two_ranks_xgmi_peer_to_peer(cuda_dev, model, dtype):
    """`bench.py --gpus 2 --comm xgmi`: the peer-to-peer communicator maps
    the other rank's buffers (on the same device here, over xGMI on a node);
    MNIST tunes its fused sync + SGD launch against the plain peer-to-peer
    all-reduce, and the replicas must end bit-identical."""
    out = _run([sys.executable, "bench.py", "--gpus", "2", "--comm", "xgmi", "--model", model,
                "--dtype", dtype, "--steps", "30", "--warmup", "5"])
    lines = _json_lines(out)
    assert len(lines) == 1, out
    c = lines[0]["config"]
    assert c["comm"] == "xgmi-p2p" and c["comm_nranks"] == 2 and c["replicas_identical"] is True
    if model == "mnist_cnn":
        tune = c["sync_tune_us_per_step"]
        # fp32 tunes the FC exchange placement too (conv2 backward / step
        # launch) and the factor gather
        want = {"xgmi", "serial"} | ({"xgmi-step", "xgmi-fac"} if dtype == "fp32" else set())
        assert tune and set(tune) == want and None not in tune.values(), tune
        assert lines[0]["final_test_accuracy"] > 50.0


def _mpipy(tmp_path, tag, *args, timeout=420):
    port = _free_port()
    ck = tmp_path / f"{tag}.npz"
    out = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                "--master-addr", "127.0.0.1", "--master-port", str(port), "mpipy.py",
                "--comm", "shm", "--synthetic", "--max-steps", "151", "--check-replicas",
                "--ckpt", str(ck), "--collective-timeout-s", "120"] + list(args), timeout=timeout)
    summ = [l for l in _json_lines(out) if "summary" in l]
    assert len(summ) == 1, out
    return out, summ[0]["summary"], ck


def _ckpt_arrays(path):
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k].copy() for k in z.files}


def test_mpipy_torchrun_grad_sync_auto_schedule_reproducible(cuda_dev, tmp_path):
    """torchrun mpipy.py, per-step gradient all-reduce: the autotuned
    schedule's run is bit-identical to a rerun that names the picked
    schedule (the tune's trial steps leave no trace), replicas are checked
    at every eval event and at the end."""
    out, s, ck = _mpipy(tmp_path, "auto", "--eval-every", "50")
    assert s["world"] == 2 and s["steps"] == 151 and s["comm"] == "host-shm"
    assert s["engine"] == "native"
    assert "Process ID: 1  training session starts!" in out
    picked = s["sync_schedule"]
    assert picked in ("buckets", "sharded", "factors"), picked
    _, s2, ck2 = _mpipy(tmp_path, "named", "--eval-every", "50", "--sync-schedule", picked)
    assert s2["sync_schedule"] == picked
    a, b = _ckpt_arrays(ck), _ckpt_arrays(ck2)
    assert sorted(a) == sorted(b)
    for k in a:
        if a[k].dtype.kind == "f":
            assert np.array_equal(a[k], b[k]), f"{k} differs between auto and named {picked}"


def test_mpipy_torchrun_param_avg(cuda_dev, tmp_path):
    """The reference's periodic weight averaging (mpipy.py:87-91) done
    right: every 50 steps ALL ranks receive the mean (the trainer checks the
    ranks' fingerprints after each average under --check-replicas)."""
    out, s, _ = _mpipy(tmp_path, "pavg", "--sync", "param_avg", "--sync-every", "50")
    assert s["world"] == 2 and s["steps"] == 151
    assert "0  process at  50 with test error:" in out
    assert "1  process at  150 with test error:" in out


def test_mpipy_torchrun_reference_quirks_root_only(cuda_dev, tmp_path):
    """--reference-quirks: root-only Gather + average of the four weights
    (Q11), padded shard (Q5), eval with dropout every step (Q8 / Q9)."""
    out, s, _ = _mpipy(tmp_path, "quirks", "--reference-quirks", "--sync", "param_avg",
                       "--sync-every", "50")
    assert s["world"] == 2 and s["steps"] == 151
    assert "0  process at  100 with test error:" in out


@pytest.mark.parametrize("sync", ["grad", "param_avg"])
def test_mpipy_torchrun_xgmi_comm(cuda_dev, tmp_path, sync):
    """`mpipy.py --comm xgmi` through torchrun: the reference's script API on
    the peer-to-peer communicator - per-step gradient sync (the fused xGMI
    schedules, tuned against the plain all-reduce) or the reference's periodic
    weight averaging (mpipy.py:87-91) over the xGMI all-reduce; replicas
    checked at every eval event and at the end."""
    extra = ["--sync", sync] + (["--sync-every", "50"] if sync == "param_avg" else [])
    out, s, _ = _mpipy(tmp_path, f"xgmi-{sync}", "--comm", "xgmi", "--eval-every", "50", *extra)
    assert s["world"] == 2 and s["steps"] == 151 and s["comm"] == "xgmi-p2p"
    if sync == "grad":
        # fp32: the FC exchange in the conv2 backward or in the step launch, the
        # factor schedule (2 ranks) or the plain all-reduce
        assert s["sync_schedule"] in ("xgmi", "xgmi-step", "xgmi-fac", "serial"), s
