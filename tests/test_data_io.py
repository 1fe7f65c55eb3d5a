"""IDX reader (Python and native C++), synthetic data, shard loading,
checkpoint round trip."""

import os

import numpy as np
import pytest
import torch

from mpi_tensorflow_amd import config as C
from mpi_tensorflow_amd.models import mnist_cnn as M
from mpi_tensorflow_amd.ops import native_available
from mpi_tensorflow_amd.utils import checkpoint
from mpi_tensorflow_amd.utils.data import load_mnist_shard, split_sizes, synthetic_rows
from mpi_tensorflow_amd.utils.idx import (error_rate, extract_data, extract_labels, read_idx_header,
                                          write_idx)


@pytest.fixture(scope="module")
def mnist_dir(tmp_path_factory):
    """Tiny MNIST-format files (gzipped IDX) - real-file code path, synthetic content."""
    d = tmp_path_factory.mktemp("mnist")
    rng = np.random.default_rng(0)
    tr = rng.integers(0, 256, size=(60000, 28, 28), dtype=np.uint8)
    write_idx(str(d / C.MNIST_FILES["train_images"]), tr)
    write_idx(str(d / C.MNIST_FILES["train_labels"]), (np.arange(60000) % 10).astype(np.uint8))
    write_idx(str(d / C.MNIST_FILES["test_images"]), tr[:10000])
    write_idx(str(d / C.MNIST_FILES["test_labels"]), (np.arange(10000) % 7).astype(np.uint8))
    return str(d), tr


def test_idx_roundtrip_and_scaling(mnist_dir):
    d, tr = mnist_dir
    path = os.path.join(d, C.MNIST_FILES["train_images"])
    magic, dims = read_idx_header(path)
    assert magic == 0x803 and dims == (60000, 28, 28)
    x = extract_data(path, 5)
    assert x.shape == (5, 28, 28, 1) and x.dtype == np.float32
    np.testing.assert_allclose(x[..., 0], (tr[:5].astype(np.float32) - 127.5) / 255.0)
    y = extract_labels(os.path.join(d, C.MNIST_FILES["train_labels"]), 12)
    assert y.dtype == np.int64 and list(y) == list(np.arange(12) % 10)


@pytest.mark.skipif(not native_available(), reason="native extension not built")
def test_native_idx_loader_matches_python(mnist_dir):
    from mpi_tensorflow_amd.ops import native

    Cn = native()
    d, tr = mnist_dir
    path = os.path.join(d, C.MNIST_FILES["train_images"])
    magic, dims = Cn.idx_header(path)
    assert magic == 0x803 and list(dims) == [60000, 28, 28]
    u8 = Cn.idx_read_u8(path, 5000, 5100)
    assert u8.shape == (100, 28, 28) and np.array_equal(u8, tr[5000:5100])
    f = Cn.idx_read_images_f32(path, 10, 20, 255.0)
    np.testing.assert_array_equal(f, extract_data(path, 20)[10:])
    with pytest.raises(RuntimeError):
        Cn.idx_read_u8(path, 0, 60001)


def test_error_rate():
    p = np.eye(10)[[1, 2, 3, 4]]
    assert error_rate(p, np.array([1, 2, 3, 4])) == 0.0
    assert error_rate(p, np.array([1, 2, 0, 0])) == 50.0


def test_synthetic_rows_are_world_independent():
    a, la = synthetic_rows("train", 900, 2100)
    b, lb = synthetic_rows("train", 1500, 1600)
    np.testing.assert_array_equal(a[600:700], b)
    np.testing.assert_array_equal(la[600:700], lb)
    assert a.min() >= -0.5 and a.max() <= 0.5
    assert len(np.unique(la)) == 10


def test_load_shard_real_files_and_padding(mnist_dir):
    d, tr = mnist_dir
    sh = load_mnist_shard(1, 2, d, synthetic=False)
    s = split_sizes(2)
    assert not sh.synthetic and sh.n_local == s.train_local == 25000
    # rank 1 train rows start at val_size + 25000 (mpipy.py:221, Scatter order)
    np.testing.assert_allclose(sh.train_x[0, ..., 0], (tr[5000 + 25000].astype(np.float32) - 127.5) / 255)
    assert sh.test_x.shape[0] == 5000 and sh.val_x.shape[0] == 2500
    q = load_mnist_shard(0, 2, d, synthetic=False, pad=True)  # quirk Q5
    assert q.n_local == 27500 and np.all(q.train_x[25000:] == 0) and np.all(q.train_y[25000:] == 0)


def test_load_shard_synthetic_when_missing(tmp_path):
    sh = load_mnist_shard(0, 8, str(tmp_path / "none"), synthetic=None)
    assert sh.synthetic and sh.n_local == 6250 and sh.test_x.shape == (1250, 28, 28, 1)


def test_checkpoint_roundtrip(tmp_path):
    lay = M.layout()
    p = torch.randn(lay.total)
    m = torch.randn(lay.total)
    path = str(tmp_path / "ck.npz")
    checkpoint.save(path, lay, p, m, 123, meta={"model": "mnist_cnn"})
    with np.load(path, allow_pickle=False) as z:
        assert z["Variable_4"].shape == (3136, 512)  # fc1_weight, TF name
        assert z["Variable_2"].shape == (5, 5, 32, 64)  # conv2 HWIO
        assert float(z["Variable_8"]) == 123.0
        assert "Variable_6/Momentum" in z.files
    p2 = torch.zeros(lay.total)
    m2 = torch.zeros(lay.total)
    step, meta = checkpoint.load(path, lay, p2, m2)
    assert step == 123 and meta["model"] == "mnist_cnn"
    for s in lay.specs:
        a, b = lay.segment(s.name)
        assert torch.equal(p2[a:b], p[a:b]) and torch.equal(m2[a:b], m[a:b])
