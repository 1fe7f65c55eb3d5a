"""Worker for tests/test_native_sync_gpu.py: N ranks share ONE GPU, each runs
the native MNIST executor with a host-staged gloo communicator (real
cross-rank data), and checks
  * buckets == a SERIAL emulation of data parallelism on rank 0 (both ranks'
    gradients computed by the same kernels, summed, one SGD with gscale 1/N):
    bit-identical params and momentum;
  * the sharded FC update and the split schedule give bit-identical params
    and (gathered) momentum to buckets;
  * switching schedules mid-run (buckets -> sharded -> buckets, what the
    startup autotune does) keeps the replicas identical to a buckets-only run
    (the FC momentum shards are gathered before leaving the sharded schedule);
  * every rank holds the same params (replica consistency);
  * with the bf16 gradient wire (--grad-comm-dtype bf16) buckets and sharded
    agree bit for bit and equal the serial emulation with the sum formed as
    bf16(sum of bf16(grad_r));
  * fp32: the factor schedule (all-gathered FC gradient factors, global FC
    gradients formed on every rank) keeps the replicas bit-identical and
    matches buckets to fp32 rounding (its FC sums run in another order), also
    when switched in and out mid-run.
Launch: torchrun --nproc-per-node 2 --master-addr 127.0.0.1 tests/helpers/native_sync_ranks.py"""
import sys

import torch
import torch.distributed as dist

from mpi_tensorflow_amd import config as C
from mpi_tensorflow_amd.ops import native, ptr, stream_handle
from mpi_tensorflow_amd.parallel import dist as D
from mpi_tensorflow_amd.parallel.comm import HostStagedComm
from mpi_tensorflow_amd.runtime.mnist_engine import NativeMnistEngine
from mpi_tensorflow_amd.utils.data import load_mnist_shard

ROWS = 4096


def _shard(rank, world, seed):
    sh = load_mnist_shard(rank, world, synthetic=True, seed=seed)
    return sh.train_x[:ROWS], sh.train_y[:ROWS]


def make(schedule, dtype, di, wire="fp32"):
    cfg = C.TrainConfig(sync_schedule=schedule, dtype=dtype, graph=False,
                        grad_comm_dtype=wire).validate()
    x, y = _shard(di.rank, di.world, cfg.seed)
    comm = HostStagedComm(di)
    eng = NativeMnistEngine(cfg, x, y, torch.device("cuda"), di.rank, di.world, comm)
    want = "buckets" if schedule == "auto" else schedule
    assert eng.grad_sync and eng.sync_schedule == want, eng.sync_schedule
    return eng


def finish(eng):
    eng.sync_optimizer_state()
    torch.cuda.synchronize()
    return eng.params.cpu(), eng.mom.cpu()


def run(schedule, dtype, steps, di, wire="fp32"):
    eng = make(schedule, dtype, di, wire)
    eng.train(steps)
    return finish(eng)


def run_switching(dtype, steps, di):
    eng = make("auto", dtype, di)
    E = native().MnistExecutor
    k = steps // 3
    eng.train(k)
    eng._set_schedule(E.SCHED_SHARDED_FC)
    assert eng.sync_schedule == "sharded"
    eng.train(k)
    eng._set_schedule(E.SCHED_BUCKETS)
    eng.train(steps - 2 * k)
    return finish(eng)


def run_factors_switching(steps, di):
    eng = make("auto", "fp32", di)
    E = native().MnistExecutor
    k = steps // 3
    eng.train(k)
    eng._set_schedule(E.SCHED_FACTORS)
    assert eng.sync_schedule == "factors"
    eng.train(k)
    eng._set_schedule(E.SCHED_BUCKETS)
    eng.train(steps - 2 * k)
    return finish(eng)


def check_factors(pb, mb, steps, di):
    out = []
    for tag, (pf, mf) in (("factors", run("factors", "fp32", steps, di)),
                          ("factors-switching", run_factors_switching(steps, di))):
        ref = pf.clone()
        dist.broadcast(ref, 0)
        assert torch.equal(ref, pf), f"{tag}: replicas diverged"
        dp = (pf - pb).abs().max().item() / pb.abs().max().item()
        dm = (mf - mb).abs().max().item() / mb.abs().max().item()
        # factors forms the global FC gradients with one K = N*B GEMM, buckets
        # sums per-rank GEMMs: a different fp32 summation order.  Through the
        # ReLU / max-pool routing (a near-zero maximum flips which element
        # receives the gradient) that grows to ~2e-4 of the largest parameter
        # after 6 steps with the Winograd conv2 (round 2, direct conv: < 1e-5)
        assert dp < 1e-3 and dm < 1e-2, f"{tag} vs buckets: rel params {dp:.2e}, momentum {dm:.2e}"
        out.append(dp)
    return max(out)


def serial(dtype, steps, world, wire="fp32"):
    """One process plays every rank: same kernels, summed grads, one SGD."""
    C_ = native()
    cfg = C.TrainConfig(dtype=dtype, graph=False).validate()
    engs = []
    for r in range(world):
        x, y = _shard(r, world, cfg.seed)
        engs.append(NativeMnistEngine(cfg, x, y, torch.device("cuda"), r, world, None))
    lead = engs[0]
    gsum = torch.empty_like(lead.grads)
    lo, hi = lead.layout.l2_range()
    assert lo == 0
    s = stream_handle()
    for _ in range(steps):
        for e in engs:
            if e is not lead:
                e.params.copy_(lead.params)
                e.step_dev.copy_(lead.step_dev)
            e.forward_backward_only()
        rnd = (lambda t: t.to(torch.bfloat16).float()) if wire == "bf16" else (lambda t: t)
        gsum.copy_(rnd(engs[0].grads))
        for e in engs[1:]:
            gsum.add_(rnd(e.grads))
        gsum.copy_(rnd(gsum))
        # lead.lr_dev was written by its head kernel from the device step
        C_.optim.sgd_momentum(ptr(lead.params), ptr(gsum), ptr(lead.mom), lead.layout.total, hi,
                              cfg.l2, cfg.momentum, 1.0 / world, ptr(lead.lr_dev), 0.0,
                              ptr(lead.step_dev), s)
    torch.cuda.synchronize()
    return lead.params.cpu(), lead.mom.cpu()


def main():
    di = D.init("cuda")
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dtype = sys.argv[2] if len(sys.argv) > 2 else "fp32"
    pb, mb = run("buckets", dtype, steps, di)
    for sched in ("sharded", "split"):
        ps, ms = run(sched, dtype, steps, di)
        assert torch.equal(pb, ps), f"{sched}: params differ: {(pb - ps).abs().max().item()}"
        assert torch.equal(mb, ms), f"{sched}: momentum differs: {(mb - ms).abs().max().item()}"
    fac_rel = check_factors(pb, mb, steps, di) if dtype == "fp32" else 0.0
    pw, mw = run_switching(dtype, steps, di)
    assert torch.equal(pb, pw), f"switching: params differ: {(pb - pw).abs().max().item()}"
    assert torch.equal(mb, mw), f"switching: momentum differs: {(mb - mw).abs().max().item()}"
    ref = pb.clone()
    dist.broadcast(ref, 0)
    assert torch.equal(ref, pb), "replicas diverged"
    assert float(pb.abs().sum()) > 0 and float(mb.abs().sum()) > 0
    if di.rank == 0:
        p1, m1 = serial(dtype, steps, di.world)
        assert torch.equal(pb, p1), f"serial emulation: params differ: {(pb - p1).abs().max().item()}"
        assert torch.equal(mb, m1), f"serial emulation: momentum differs: {(mb - m1).abs().max().item()}"
    # bf16 gradient wire
    pbb, mbb = run("buckets", dtype, steps, di, "bf16")
    psb, msb = run("sharded", dtype, steps, di, "bf16")
    assert torch.equal(pbb, psb) and torch.equal(mbb, msb), "bf16 wire: sharded != buckets"
    assert not torch.equal(pbb, pb), "bf16 wire left the update unchanged"
    if di.rank == 0:
        p2, m2 = serial(dtype, steps, di.world, "bf16")
        assert torch.equal(pbb, p2), f"bf16 wire vs serial: params differ: {(pbb - p2).abs().max().item()}"
        assert torch.equal(mbb, m2), f"bf16 wire vs serial: momentum differs: {(mbb - m2).abs().max().item()}"
        rel = ((pbb - pb).norm() / pb.norm()).item()
        assert rel < 1e-2, f"bf16 wire drifted from fp32: rel {rel}"
        print(f"NATIVE_SYNC_OK world={di.world} steps={steps} dtype={dtype} bf16-wire-rel={rel:.2e} "
              f"factors-rel={fac_rel:.2e}", flush=True)
    D.barrier()
    D.shutdown()


if __name__ == "__main__":
    main()
