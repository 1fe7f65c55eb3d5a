import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

os.environ.setdefault("OMP_NUM_THREADS", "4")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the native HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def cuda_dev():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mpi_tensorflow_amd.ops import require_native

    require_native()  # GPU tests must run the native path, never a fallback
    return torch.device("cuda:0")


@pytest.fixture(autouse=True)
def _reset_conv_mode():
    """Engines set the process-wide conv operand mode (Fn.set_conv_bf16);
    restore fp32 after every test so later tests start from the default."""
    yield
    try:
        from mpi_tensorflow_amd.ops import functional as Fn
    except Exception:  # noqa: BLE001 - CPU-only collection without the package deps
        return
    Fn.set_conv_bf16(False)
