"""Spec-layer unit tests (CPU): constants, sizing/sharding math, LR schedule,
dropout RNG, flat layout, log formats.  Expected values are derived from the
reference script (/root/reference/mpipy.py line refs in each test)."""

import numpy as np
import pytest

from mpi_tensorflow_amd import config as C
from mpi_tensorflow_amd.models import mnist_cnn as M
from mpi_tensorflow_amd.utils import rng
from mpi_tensorflow_amd.utils.data import (batch_offset, local_train_rows, num_syncs, shard_ranges,
                                           split_sizes, steps_per_run)
from mpi_tensorflow_amd.utils.logging import progress_line, start_line
from mpi_tensorflow_amd.utils.schedule import learning_rate


def test_reference_constants():
    # mpipy.py:17-21, :57, :60-65, :87, :166
    assert (C.ITERATION, C.IMAGE_SIZE, C.BATCH_SIZE, C.NUM_CHANNEL) == (2, 28, 64, 10)
    assert (C.BASE_LR, C.LR_DECAY, C.MOMENTUM, C.L2_COEF) == (0.01, 0.95, 0.9, 5e-4)
    assert C.SYNC_EVERY == 50 and C.DROPOUT_KEEP == 0.5 and C.SEED == 1
    assert C.DATA_URL.endswith("/mnist/")


def test_cli_defaults_and_overrides():
    cfg = C.config_from_args([])
    assert cfg.batch_size == 64 and cfg.epochs == 2 and cfg.sync == "grad"
    assert not cfg.reference_quirks and cfg.effective_eval_every() == 50
    cfg = C.config_from_args(["--reference-quirks", "--sync", "param_avg", "--batch-size", "32"])
    assert cfg.pad_train_shard and cfg.eval_dropout and cfg.root_only_average
    assert cfg.same_seed_all_ranks and cfg.effective_eval_every() == 1
    with pytest.raises(SystemExit):
        C.config_from_args(["--model", "vgg"])


@pytest.mark.parametrize("P,tr,ts,val", [(1, 55000, 10000, 5000), (2, 55000, 10000, 5000),
                                         (3, 54999, 9999, 4998), (8, 55000, 10000, 5000),
                                         (7, 54999, 9996, 4998)])
def test_split_sizes(P, tr, ts, val):
    s = split_sizes(P)  # mpipy.py:211-213
    assert (s.tr_size, s.ts_size, s.val_size) == (tr, ts, val)
    assert s.train_local * P == tr - val
    assert s.train_local_padded == tr // P


@pytest.mark.parametrize("P,padded,fixed", [(1, 1718, 1562), (2, 859, 781), (4, 429, 390),
                                            (8, 214, 195)])
def test_steps_per_run(P, padded, fixed):
    s = split_sizes(P)  # mpipy.py:79 with N_local = tr_size//P (quirk Q5) or the real rows
    assert steps_per_run(local_train_rows(s, pad=True)) == padded
    assert steps_per_run(local_train_rows(s, pad=False)) == fixed


def test_shards_disjoint_and_cover():
    for P in (1, 2, 4, 8):
        s = split_sizes(P)
        tr = [shard_ranges(s, r)["train"] for r in range(P)]
        assert tr[0][0] == s.val_size and tr[-1][1] == s.tr_size
        assert all(tr[i][1] == tr[i + 1][0] for i in range(P - 1))
        ts = [shard_ranges(s, r)["test"] for r in range(P)]
        assert ts[0][0] == 0 and ts[-1][1] == s.ts_size
    with pytest.raises(ValueError):
        shard_ranges(split_sizes(2), 2)


def test_batch_offset_and_syncs():
    # mpipy.py:80: (step*64) % (N - 64)
    n = 50000
    assert batch_offset(0, n) == 0
    assert batch_offset(780, n) == (780 * 64) % (n - 64)
    assert all(0 <= batch_offset(s, n) <= n - 64 for s in range(0, 5000, 37))
    assert num_syncs(1718) == 34 and num_syncs(214) == 4


def test_learning_rate_staircase():
    n = 50000
    assert learning_rate(0, n) == pytest.approx(0.01)
    last0 = n // 64  # last step whose step*64 < n
    assert learning_rate(last0, n) == pytest.approx(0.01)
    assert learning_rate(last0 + 1, n) == pytest.approx(0.0095)
    assert learning_rate(2 * n // 64 + 1, n) == pytest.approx(0.01 * 0.95 ** 2, rel=1e-6)


def test_dropout_rng_properties():
    k0 = rng.dropout_key(1, 0, 0)
    assert k0 == rng.dropout_key(1, 0, 0)
    keys = {rng.dropout_key(1, r, s) for r in range(4) for s in range(50)}
    assert len(keys) == 200
    m = rng.keep_mask_np(k0, 200000, 0.5)
    assert abs(m.mean() - 0.5) < 0.01
    m2 = rng.keep_mask_np(rng.dropout_key(1, 0, 1), 200000, 0.5)
    assert abs((m & m2).mean() - 0.25) < 0.01  # independent across steps
    assert rng.keep_mask_np(k0, 1000, 1.0).all()


def test_flat_layout():
    lay = M.layout()
    assert lay.numel == 1663370
    assert all(o % 64 == 0 for o in lay.offsets.values())
    b = lay.buckets()
    assert len(b) == 2 and b[0][0] == 0 and b[1][1] == lay.total
    # bucket 1 = FC params, 97 % of the bytes
    assert (b[0][1] - b[0][0]) / lay.total > 0.96
    lo, hi = lay.l2_range()
    assert (lo, hi) == b[0]
    names = lay.tf_names()
    assert names["conv1_weight"] == "Variable" and names["fc2_bias"] == "Variable_7"


def test_init_params_deterministic_and_shaped():
    import torch

    lay = M.layout()
    a = torch.zeros(lay.total)
    b = torch.zeros(lay.total)
    M.init_params(a, lay, seed=1)
    M.init_params(b, lay, seed=1)
    assert torch.equal(a, b)
    v = lay.views(a)
    assert v["conv1_bias"].abs().sum() == 0
    assert torch.allclose(v["fc1_bias"], torch.full((512,), 0.1))
    w = v["fc1_weight"]
    assert w.abs().max() <= 0.2 + 1e-6 and abs(w.std().item() - 0.088) < 0.005


def test_log_formats_match_reference():
    # mpipy.py:77 and :88 as printed by Python's print()
    assert start_line(0) == "Process ID: 0  training session starts!"
    assert progress_line(3, 50, 1.234) == "3  process at  50 with test error: 1.2%"
