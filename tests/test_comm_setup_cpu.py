"""One communicator set-up for bench.py and the mpipy.py Trainer
(parallel/setup.py), and the exactness-check data of the xGMI gate
(parallel/comm.py xgmi_exactness_check).  The reference has one
communicator, MPI.COMM_WORLD (/root/reference/mpipy.py:208-210)."""
import numpy as np
import pytest
import torch

import bench
from mpi_tensorflow_amd import config as C
from mpi_tensorflow_amd.parallel import comm as CM
from mpi_tensorflow_amd.parallel import setup as SU
from mpi_tensorflow_amd.runtime import trainer as TR


def test_xgmi_candidate_rule():
    base = C.TrainConfig().validate()
    assert SU.wants_xgmi_candidate(base, "rccl-native")
    assert not SU.wants_xgmi_candidate(base, "rccl-native", no_xgmi=True)
    assert not SU.wants_xgmi_candidate(base, "host-shm")  # ranks share GPUs
    assert not SU.wants_xgmi_candidate(base, "torch-gloo")
    assert SU.wants_xgmi_candidate(C.TrainConfig(model="lenet5").validate(), "rccl-native")
    for kw in (dict(comm="rccl"), dict(model="resnet18"), dict(sync="param_avg"), dict(no_xgmi=True)):
        cfg = C.TrainConfig(**kw).validate()
        assert not SU.wants_xgmi_candidate(cfg, "rccl-native", no_xgmi=cfg.no_xgmi), kw
    assert SU.wants_comm(base, 2) and not SU.wants_comm(base, 1)
    assert not SU.wants_comm(C.TrainConfig(sync="none").validate(), 8)


def _record(monkeypatch, module):
    seen = []

    def fake(di, device, cfg, no_xgmi=False, xgmi_timeout_s=20.0):
        seen.append((cfg, no_xgmi))
        return SU.CommSet()

    monkeypatch.setattr(module, "setup_comms", fake)
    return seen


@pytest.mark.parametrize("extra", [[], ["--no-xgmi"]])
def test_bench_and_trainer_build_the_same_candidate_set(monkeypatch, extra):
    """bench.py and the Trainer both go through setup_comms with configs that
    take the same xGMI decision for the same flags."""
    seen_t = _record(monkeypatch, TR)
    cfg_t = C.config_from_args(["--max-steps", "1", "--eval-every", "0", "--quiet"] + extra)
    tr = TR.Trainer(cfg_t)
    tr.watchdog.stop()
    seen_b = _record(monkeypatch, SU)  # bench imports it from the module at run time
    rc = bench.main(["--steps", "1", "--warmup", "0", "--no-eval", "--prewarm-ms", "0"] + extra)
    assert rc == 0
    assert len(seen_t) == 1 and len(seen_b) == 1
    (ct, nt), (cb, nb) = seen_t[0], seen_b[0]
    for kind in ("rccl-native", "host-shm", "torch-gloo"):
        assert (SU.wants_xgmi_candidate(ct, kind, nt) == SU.wants_xgmi_candidate(cb, kind, nb)), kind
    assert SU.wants_xgmi_candidate(cb, "rccl-native", nb) == (extra == [])
    for f in ("model", "comm", "sync", "no_xgmi", "sync_schedule", "dtype"):
        assert getattr(ct, f) == getattr(cb, f), f
    assert SU.comm_capacity_bytes(ct) == SU.comm_capacity_bytes(cb)
    assert TR.comm_capacity_bytes is SU.comm_capacity_bytes


@pytest.mark.parametrize("n", [2, 3, 7, 8])
def test_exactness_pattern_sums_are_exact_and_ranks_differ(n):
    count = 61_440
    parts = [CM.exact_pattern(r, 3, count) for r in range(n)]
    for p in parts:
        assert float(p.abs().max()) <= 125 and torch.equal(p, p.round())
    want = CM.exact_sum(n, 3, count)
    # any summation order gives the same bits (exact integers in fp32)
    fwd = torch.zeros(count)
    for p in parts:
        fwd += p
    rev = torch.zeros(count)
    for p in reversed(parts):
        rev += p
    assert torch.equal(fwd, want) and torch.equal(rev, want)
    # a rank left out of the sum changes ~250 of 251 elements
    for k in range(n):
        miss = want - parts[k]
        frac = float((miss != want).double().mean())
        assert frac > 0.99, (k, frac)
    # rounds use fresh data: a read of the previous round's bytes fails
    assert float((CM.exact_pattern(0, 3, count) != CM.exact_pattern(0, 5, count)).double().mean()) > 0.99
    assert np.all(np.diff([CM.exact_pattern(r, 0, 8)[0].item() for r in range(n)]) != 0)


def test_lenet_xgmi_mode_config_and_bench_flags():
    """LeNet-5's xGMI sync mode: validated by TrainConfig (default pull), and
    bench.py's --xgmi-mode / --xgmi-push map onto it."""
    assert C.TrainConfig().validate().xgmi_mode == "pull"
    for m in C.XGMI_MODES:
        assert C.TrainConfig(xgmi_mode=m).validate().xgmi_mode == m
    with pytest.raises(ValueError):
        C.TrainConfig(xgmi_mode="ring").validate()
    assert bench.parse([]).xgmi_mode == "pull"
    assert bench.parse(["--xgmi-mode", "two-phase"]).xgmi_mode == "two-phase"
    a = bench.parse(["--xgmi-push"])
    assert a.xgmi_push and ("push" if a.xgmi_push else a.xgmi_mode) == "push"
    a = bench.parse(["--bn-fused", "on", "--bn-fused-bpc", "3"])
    assert a.bn_fused == "on" and a.bn_fused_bpc == 3
