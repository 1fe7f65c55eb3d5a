"""IDX (MNIST) file reader/writer and the tutorial helpers the reference imports.

The reference imports `extract_data`, `extract_labels` and `error_rate` from
the TensorFlow tutorial's `convolutional.py` (`/root/reference/mpipy.py:12`,
used at `:215-218` and `:86`); that file is not part of the reference, so the
semantics implemented here are the tutorial's public behaviour:

* `extract_data(path, n)`   -> float32 [n, 28, 28, 1], (pixel - 127.5) / 255
* `extract_labels(path, n)` -> int64 [n]
* `error_rate(pred, labels)` -> 100 - 100 * mean(argmax(pred, 1) == labels)

A native C++ reader (`csrc/idx_loader.cpp`, exposed as `_C.idx_read`) does the
same parse with zlib; this pure-Python version is the fallback and the oracle
the native one is tested against.
"""

from __future__ import annotations

import gzip
import os
import struct
from typing import Tuple

import numpy as np

from ..config import IMAGE_SIZE, PIXEL_DEPTH

IDX_IMAGES_MAGIC = 0x00000803  # ubyte, 3 dims
IDX_LABELS_MAGIC = 0x00000801  # ubyte, 1 dim


def _open(path: str):
    with open(path, "rb") as f:
        head = f.read(2)
    return gzip.open(path, "rb") if head == b"\x1f\x8b" else open(path, "rb")


def read_idx_header(path: str) -> Tuple[int, Tuple[int, ...]]:
    """Returns (magic, dims) of an IDX file (gzipped or raw)."""
    with _open(path) as f:
        magic = struct.unpack(">I", f.read(4))[0]
        ndim = magic & 0xFF
        dims = struct.unpack(">" + "I" * ndim, f.read(4 * ndim))
    return magic, dims


def read_idx_raw(path: str, count: int) -> np.ndarray:
    """Reads the first `count` records of an IDX file as uint8 with the
    record shape given by its header."""
    magic, dims = read_idx_header(path)
    if (magic >> 8) != 0x08:
        raise ValueError(f"{path}: unsupported IDX element type 0x{magic:08x}")
    if count > dims[0]:
        raise ValueError(f"{path}: asked for {count} records, file has {dims[0]}")
    rec = int(np.prod(dims[1:])) if len(dims) > 1 else 1
    with _open(path) as f:
        f.read(4 + 4 * len(dims))
        buf = f.read(rec * count)
    if len(buf) != rec * count:
        raise ValueError(f"{path}: truncated file")
    return np.frombuffer(buf, dtype=np.uint8).reshape((count,) + tuple(dims[1:]))


def extract_data(filename: str, num_images: int) -> np.ndarray:
    """Images -> float32 [n, 28, 28, 1] in [-0.5, 0.5] (tutorial semantics)."""
    raw = read_idx_raw(filename, num_images).astype(np.float32)
    data = (raw - PIXEL_DEPTH / 2.0) / PIXEL_DEPTH
    return data.reshape(num_images, IMAGE_SIZE, IMAGE_SIZE, 1)


def extract_labels(filename: str, num_images: int) -> np.ndarray:
    """Labels -> int64 [n]."""
    return read_idx_raw(filename, num_images).astype(np.int64).reshape(num_images)


def error_rate(predictions: np.ndarray, labels: np.ndarray) -> float:
    """Percentage of rows whose argmax differs from the label."""
    predictions = np.asarray(predictions)
    labels = np.asarray(labels).astype(np.int64)
    correct = np.sum(np.argmax(predictions, 1) == labels)
    return 100.0 - (100.0 * correct / predictions.shape[0])


def write_idx(path: str, array: np.ndarray, gz: bool = True) -> None:
    """Writes a uint8 array as an IDX file (used for fixtures and tests)."""
    array = np.ascontiguousarray(array, dtype=np.uint8)
    magic = 0x00000800 | array.ndim
    header = struct.pack(">I", magic) + struct.pack(">" + "I" * array.ndim, *array.shape)
    opener = gzip.open if gz else open
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with opener(path, "wb") as f:
        f.write(header)
        f.write(array.tobytes())
