"""Worker for tests/test_native_sync_gpu.py: N ranks share ONE GPU and train
a generic model (LeNet-5 / ResNet-18) with per-step gradient all-reduce over a
host-staged gloo communicator, so the backward-overlapped bucketed all-reduce
(parallel/overlap.py: grad hooks -> bucket events -> comm stream) moves real
cross-rank sums.  Rank 0 then replays the same steps SERIALLY (every rank's
forward/backward on the same kernels, grads summed, one SGD with gscale 1/N)
and the params must be bit-identical; all ranks must hold the same params.
MODEL "lenet5-native" runs the fused LeNet-5 executor (runtime/lenet_engine.py)
instead, whose single flat-gradient all-reduce goes through the same comm.
WIRE "bf16" (optional 4th argument) uses the bf16 gradient wire
(--grad-comm-dtype bf16); the serial emulation then sums bf16(grad_r) and
rounds the sum to bf16.
Launch: torchrun --nproc-per-node 2 ... generic_sync_ranks.py MODEL STEPS BATCH [WIRE]"""
import sys

import numpy as np
import torch
import torch.distributed as dist

from mpi_tensorflow_amd import config as C
from mpi_tensorflow_amd.models.generic import model_input_shape
from mpi_tensorflow_amd.parallel import dist as D
from mpi_tensorflow_amd.parallel.comm import HostStagedComm
from mpi_tensorflow_amd.ops import native, ptr, stream_handle
from mpi_tensorflow_amd.runtime.generic_engine import GenericEngine
from mpi_tensorflow_amd.runtime.lenet_engine import NativeLenetEngine
from mpi_tensorflow_amd.utils.data import synthetic_images_torch


def shard(model, rank, rows, seed):
    x, y = synthetic_images_torch(rows, model_input_shape(model), seed=seed, start=rank * rows)
    return x.numpy(), y.numpy()


def main():
    model = sys.argv[1]
    fused = model == "lenet5-native"
    if fused:
        model = "lenet5"
    Eng = NativeLenetEngine if fused else GenericEngine
    steps = int(sys.argv[2])
    B = int(sys.argv[3])
    wire = sys.argv[4] if len(sys.argv) > 4 else "fp32"
    rows = 4 * B
    di = D.init("cuda")
    dev = torch.device("cuda")
    cfg = C.TrainConfig(model=model, batch_size=B, graph=False, grad_comm_dtype=wire).validate()
    x, y = shard(model, di.rank, rows, cfg.seed)
    eng = Eng(cfg, x, y, dev, di.rank, di.world, HostStagedComm(di))
    assert eng.grad_sync
    nb = 1 if fused else len(eng.bucketer.slices)
    eng.train(steps)
    torch.cuda.synchronize()
    p = eng.params.detach().cpu()
    ref = p.clone()
    dist.broadcast(ref, 0)
    assert torch.equal(ref, p), "replicas diverged"
    if di.rank == 0:
        engs = [Eng(cfg, *shard(model, r, rows, cfg.seed), dev, r, di.world, None)
                for r in range(di.world)]
        lead = engs[0]
        for _ in range(steps):
            for e in engs:
                if e is not lead:
                    e.params.data.copy_(lead.params.data)
                    e.step_dev.copy_(lead.step_dev)
                if fused:
                    e.forward_backward_only()
                else:
                    e.forward_backward_gpu()
            if wire == "bf16":
                gs = sum(e.grads.to(torch.bfloat16).float() for e in engs)
                lead.grads.copy_(gs.to(torch.bfloat16).float())
            else:
                for e in engs[1:]:
                    lead.grads.add_(e.grads)
            if fused:  # the flat SGD the executor runs after its all-reduce
                native().optim.sgd_momentum(ptr(lead.params), ptr(lead.grads), ptr(lead.mom),
                                            lead.layout.total, 0, 0.0, cfg.momentum,
                                            1.0 / di.world, ptr(lead.lr_dev), 0.0,
                                            ptr(lead.step_dev), stream_handle())
            else:
                lead.update_gpu(1.0 / di.world)
        torch.cuda.synchronize()
        q = lead.params.detach().cpu()
        d = (p - q).abs().max().item()
        assert torch.equal(p, q), f"serial emulation differs by {d}"
        assert np.isfinite(p.numpy()).all()
        print(f"GENERIC_SYNC_OK model={sys.argv[1]} world={di.world} buckets={nb} steps={steps} "
              f"wire={wire}", flush=True)
    D.barrier()
    D.shutdown()


if __name__ == "__main__":
    main()
