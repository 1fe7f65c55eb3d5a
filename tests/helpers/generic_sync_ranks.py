"""Worker for tests/test_native_sync_gpu.py: N ranks share ONE GPU and train
a generic model (LeNet-5 / ResNet-18) with per-step gradient all-reduce over a
host-staged gloo communicator, so the backward-overlapped bucketed all-reduce
(parallel/overlap.py: grad hooks -> bucket events -> comm stream) moves real
cross-rank sums.  Rank 0 then replays the same steps SERIALLY (every rank's
forward/backward on the same kernels, grads summed, one SGD with gscale 1/N)
and the params must be bit-identical; all ranks must hold the same params.
Launch: torchrun --nproc-per-node 2 ... generic_sync_ranks.py MODEL STEPS BATCH"""
import sys

import numpy as np
import torch
import torch.distributed as dist

from mpi_tensorflow_amd import config as C
from mpi_tensorflow_amd.models.generic import model_input_shape
from mpi_tensorflow_amd.parallel import dist as D
from mpi_tensorflow_amd.parallel.comm import HostStagedComm
from mpi_tensorflow_amd.runtime.generic_engine import GenericEngine
from mpi_tensorflow_amd.utils.data import synthetic_images_torch


def shard(model, rank, rows, seed):
    x, y = synthetic_images_torch(rows, model_input_shape(model), seed=seed, start=rank * rows)
    return x.numpy(), y.numpy()


def main():
    model = sys.argv[1]
    steps = int(sys.argv[2])
    B = int(sys.argv[3])
    rows = 4 * B
    di = D.init("cuda")
    dev = torch.device("cuda")
    cfg = C.TrainConfig(model=model, batch_size=B, graph=False).validate()
    x, y = shard(model, di.rank, rows, cfg.seed)
    eng = GenericEngine(cfg, x, y, dev, di.rank, di.world, HostStagedComm(di))
    assert eng.bucketer is not None
    nb = len(eng.bucketer.slices)
    eng.train(steps)
    torch.cuda.synchronize()
    p = eng.params.detach().cpu()
    ref = p.clone()
    dist.broadcast(ref, 0)
    assert torch.equal(ref, p), "replicas diverged"
    if di.rank == 0:
        engs = [GenericEngine(cfg, *shard(model, r, rows, cfg.seed), dev, r, di.world, None)
                for r in range(di.world)]
        lead = engs[0]
        for _ in range(steps):
            for e in engs:
                if e is not lead:
                    e.params.data.copy_(lead.params.data)
                    e.step_dev.copy_(lead.step_dev)
                e.forward_backward_gpu()
            for e in engs[1:]:
                lead.grads.add_(e.grads)
            lead.update_gpu(1.0 / di.world)
        torch.cuda.synchronize()
        q = lead.params.detach().cpu()
        d = (p - q).abs().max().item()
        assert torch.equal(p, q), f"serial emulation differs by {d}"
        assert np.isfinite(p.numpy()).all()
        print(f"GENERIC_SYNC_OK model={model} world={di.world} buckets={nb} steps={steps}",
              flush=True)
    D.barrier()
    D.shutdown()


if __name__ == "__main__":
    main()
