"""Worker for tests/test_native_sync_gpu.py: N ranks share ONE GPU, each runs
the native MNIST executor with a host-staged gloo communicator, once with the
bucketed all-reduce schedule and once with the sharded FC update, and checks
  * both schedules give bit-identical params (same sums, same elementwise SGD),
  * the gathered momentum is identical too,
  * every rank holds the same params (replica consistency).
Launch: torchrun --nproc-per-node 2 --master-addr 127.0.0.1 tests/helpers/native_sync_ranks.py"""
import sys

import torch
import torch.distributed as dist

from mpi_tensorflow_amd import config as C
from mpi_tensorflow_amd.parallel import dist as D
from mpi_tensorflow_amd.parallel.comm import HostStagedComm
from mpi_tensorflow_amd.runtime.mnist_engine import NativeMnistEngine
from mpi_tensorflow_amd.utils.data import load_mnist_shard


def run(schedule: str, dtype: str, steps: int, di):
    cfg = C.TrainConfig(sync_schedule=schedule, dtype=dtype, graph=False).validate()
    shard = load_mnist_shard(di.rank, di.world, synthetic=True, seed=cfg.seed)
    comm = HostStagedComm(di)
    eng = NativeMnistEngine(cfg, shard.train_x[:4096], shard.train_y[:4096],
                            torch.device("cuda"), di.rank, di.world, comm)
    assert eng.grad_sync and eng.sync_schedule == schedule, eng.sync_schedule
    eng.train(steps)
    eng.sync_optimizer_state()
    torch.cuda.synchronize()
    return eng.params.cpu(), eng.mom.cpu()


def main():
    di = D.init("cuda")
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dtype = sys.argv[2] if len(sys.argv) > 2 else "fp32"
    pb, mb = run("buckets", dtype, steps, di)
    for sched in ("sharded", "split"):
        ps, ms = run(sched, dtype, steps, di)
        assert torch.equal(pb, ps), f"{sched}: params differ: {(pb - ps).abs().max().item()}"
        assert torch.equal(mb, ms), f"{sched}: momentum differs: {(mb - ms).abs().max().item()}"
    ref = pb.clone()
    dist.broadcast(ref, 0)
    assert torch.equal(ref, pb), "replicas diverged"
    assert float(pb.abs().sum()) > 0 and float(mb.abs().sum()) > 0
    if di.rank == 0:
        print(f"NATIVE_SYNC_OK world={di.world} steps={steps} dtype={dtype}", flush=True)
    D.barrier()
    D.shutdown()


if __name__ == "__main__":
    main()
