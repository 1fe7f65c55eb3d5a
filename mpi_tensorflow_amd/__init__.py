"""mpi_tensorflow_amd - an MI355X-native (gfx950 / CDNA4) data-parallel CNN
training framework with the capabilities of youzhenfei1995/mpi-Tensorflow.

Layout:
  config.py        reference defaults + CLI (mpipy.py:14-21, :57-66, :87)
  models/          MNIST CNN (reference), LeNet-5, ResNet-18
  ops/             native extension loader (+ autograd ops for generic models)
  parallel/        rank discovery, RCCL communicator, flat buffers, DP sync
  runtime/         step engines (fused HIP kernels + hipGraph), trainer
  utils/           IDX reader, data sharding/synthetic data, RNG, LR, ckpt
  csrc/            HIP kernels (gfx950) + C++ runtime (executor, RCCL, IDX)

The one-script entry point is `mpipy.py` at the repository root.
"""

__version__ = "0.1.0"

from . import config  # noqa: F401
