"""One-script API, same name and defaults as the reference's `mpipy.py`.

Reference usage: `mpirun -np P python mpipy.py` (no flags; every knob is a
module global, /root/reference/mpipy.py:14-21).  Here:

    python mpipy.py                                  # 1 process (GPU 0 or CPU)
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 mpipy.py
    mpirun -np 8 python mpipy.py                     # OMPI_/PMI_ env honoured

with optional overrides (see --help): --epochs, --batch-size, --model
{mnist_cnn,lenet5,resnet18}, --sync {grad,param_avg,none}, --sync-every,
--eval-every, --synthetic, --ckpt/--resume, --metrics-jsonl,
--reference-quirks.  Log lines keep the reference's exact formats.
"""

from __future__ import annotations

import json
import os
import sys

# mpipy.py:14-15 set these before running; keep them for parity (TF-only
# knobs, harmless here).
os.environ.setdefault("TF_CPP_MIN_LOG_LEVEL", "2")
os.environ.setdefault("MPI_OPTIMAL_PATH", "1")

from mpi_tensorflow_amd.config import (BATCH_SIZE, DATA_URL, IMAGE_SIZE, ITERATION,  # noqa: E402,F401
                                       NUM_CHANNEL, config_from_args)


def main(argv=None) -> int:
    cfg = config_from_args(argv)
    from mpi_tensorflow_amd.runtime.trainer import Trainer

    tr = Trainer(cfg)
    summary = tr.run()
    if tr.rank == 0 and not cfg.quiet:
        print(json.dumps({"summary": summary.as_dict()}, sort_keys=True))
        sys.stdout.flush()
    from mpi_tensorflow_amd.parallel import dist as D

    D.barrier()
    D.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
