"""Native op library loader.

`mpi_tensorflow_amd._C` is the in-tree hipcc-built extension (gfx950 code
objects, RCCL loader, IDX reader, step executor).  It is imported AFTER
torch so that it binds to the HIP runtime the PyTorch-ROCm wheel loaded
(same soname, one runtime per process).

On a machine with a GPU the native path is mandatory: `require_native()`
raises instead of silently falling back to PyTorch ops, so a GPU test or
bench can never "pass" on an eager fallback.
"""

from __future__ import annotations

import os
from typing import Optional

import torch  # noqa: F401  (must precede the extension import)

_C = None
_ERR: Optional[BaseException] = None


def _load():
    global _C, _ERR
    if _C is not None or _ERR is not None:
        return
    try:
        from .. import _C as mod  # type: ignore

        _C = mod
    except BaseException as e:  # ImportError, OSError (missing runtime)
        _ERR = e


def native_available() -> bool:
    _load()
    return _C is not None


def native():
    """The extension module; raises a descriptive error when it is missing."""
    _load()
    if _C is None:
        raise RuntimeError(
            "mpi_tensorflow_amd native extension (_C) is not built or failed to load "
            f"({_ERR!r}); run `python -m mpi_tensorflow_amd.build_ext`"
        )
    return _C


def require_native():
    """Native path is required whenever a GPU is present (fail loudly)."""
    return native()


def torch_lib_dir() -> str:
    return os.path.join(os.path.dirname(torch.__file__), "lib")


def stream_handle(stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def ptr(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else int(t.data_ptr())
