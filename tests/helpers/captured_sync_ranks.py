"""Worker for tests/test_captured_sync_gpu.py: 2 ranks share ONE GPU and run
the CAPTURED (hipGraph-replayed) gradient-sync schedules with real
cross-rank data through the shared-memory communicator (csrc/shm_comm.h:
D2H copy -> host-function exchange -> H2D copy, all captured).  Every result
is compared bit for bit with the eager host-staged gloo communicator
(parallel/comm.py HostStagedComm) running the same schedule, and/or with a
serial emulation of data parallelism on rank 0.

usage: captured_sync_ranks.py SCENARIO [DTYPE]
  mnist DTYPE   - native MNIST executor: buckets / sharded / split (/ factors, defer,
                  fp32) captured vs eager; bf16 gradient wire; the
                  auto-tune (side-effect free, then the chosen schedule) and
                  a captured switching sequence; replica fingerprints
  param_avg     - the reference's periodic weight averaging (mpipy.py:87-91,
                  :95-153) on the native engine: all-ranks average and the
                  root-only quirk (Q11), through the shm communicator
  generic MODEL - ResNet-18 (B=4, 2-step graphs after the eager warm-up) or
                  the fused LeNet-5 executor with captured bucketed sync vs
                  the serial emulation
  xgmi DTYPE    - the xGMI peer-to-peer communicator over IPC-mapped buffers
                  of the two processes (csrc/xgmi_comm.h): its all-reduce and
                  segment gather vs gloo, and the captured fused sync + SGD
                  schedule (SCHED_XGMI) and its plain all-reduce schedule vs the
                  eager buckets schedule, bit for bit
"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from mpi_tensorflow_amd import config as C  # noqa: E402
from mpi_tensorflow_amd.ops import native, ptr, stream_handle  # noqa: E402
from mpi_tensorflow_amd.parallel import dist as D  # noqa: E402
from mpi_tensorflow_amd.parallel.comm import HostStagedComm, ShmDeviceComm  # noqa: E402
from mpi_tensorflow_amd.parallel.sync import (average_params, average_params_root_only,  # noqa: E402
                                              replicas_identical, REFERENCE_AVERAGED)
from mpi_tensorflow_amd.runtime.mnist_engine import NativeMnistEngine  # noqa: E402
from mpi_tensorflow_amd.runtime.trainer import comm_capacity_bytes  # noqa: E402

import native_sync_ranks as NS  # noqa: E402

STEPS, G = 7, 3  # 2 full 3-step graphs + a 1-step remainder graph


def mnist_engine(di, schedule, dtype, comm_kind, wire="fp32", graph=True, sync="grad"):
    cfg = C.TrainConfig(sync_schedule=schedule, dtype=dtype, graph=graph, graph_steps=G,
                        grad_comm_dtype=wire, sync=sync).validate()
    x, y = NS._shard(di.rank, di.world, cfg.seed)
    comm = (HostStagedComm(di) if comm_kind == "eager"
            else ShmDeviceComm(di, comm_capacity_bytes(cfg), timeout_s=60.0))
    eng = NativeMnistEngine(cfg, x, y, torch.device("cuda"), di.rank, di.world, comm)
    if sync == "grad":
        assert eng.use_graph == (comm_kind != "eager")
    return eng


def finish(eng):
    eng.sync_optimizer_state()
    torch.cuda.synchronize()
    assert replicas_identical(eng.params) and replicas_identical(eng.mom), "replicas differ"
    return eng.params.cpu(), eng.mom.cpu()


def same(a, b, what):
    pa, ma = a
    pb, mb = b
    assert torch.equal(pa, pb), f"{what}: params differ by {(pa - pb).abs().max().item():.3e}"
    assert torch.equal(ma, mb), f"{what}: momentum differs by {(ma - mb).abs().max().item():.3e}"


def run_fixed(di, sched, dtype, kind, wire="fp32"):
    eng = mnist_engine(di, sched, dtype, kind, wire)
    assert eng.sync_schedule == sched, (eng.sync_schedule, sched)
    eng.train(STEPS)
    return finish(eng), eng


def scenario_mnist(di, dtype):
    scheds = ["buckets", "sharded", "split", "serial"] + (
        ["factors", "defer"] if dtype == "fp32" else [])
    eager = {}
    for sched in scheds:
        e, _ = run_fixed(di, sched, dtype, "eager")
        c, eng = run_fixed(di, sched, dtype, "shm")
        same(c, e, f"{sched} captured vs eager")
        eager[sched] = e
        assert len(eng._graphs) == 2, "expected the 3-step and the 1-step graph"
    for sched in ("sharded", "split", "serial") + (("defer",) if dtype == "fp32" else ()):
        same(eager[sched], eager["buckets"], f"{sched} vs buckets")  # bit-identical schedules
    # bf16 gradient wire, captured
    for sched in ("buckets", "sharded"):
        e, _ = run_fixed(di, sched, dtype, "eager", "bf16")
        c, _ = run_fixed(di, sched, dtype, "shm", "bf16")
        same(c, e, f"bf16 wire {sched} captured vs eager")
    # auto-tune: side-effect free, then trains with the schedule it picked
    eng = mnist_engine(di, "auto", dtype, "shm")
    p0, m0 = eng.params.clone(), eng.mom.clone()
    trial = eng.tune_schedule()
    assert trial > 0 and eng.step == 0 and int(eng.step_dev.item()) == 0
    assert torch.equal(eng.params, p0) and torch.equal(eng.mom, m0), "tune changed the state"
    picked = eng.sync_schedule
    eng.train(STEPS)
    ref, _ = run_fixed(di, picked, dtype, "shm")
    same(finish(eng), ref, f"auto (picked {picked}) vs fixed {picked}")
    # captured switching sequence (what a re-tune does mid-run) vs the same
    # sequence eagerly
    E = native().MnistExecutor
    seq = [E.SCHED_BUCKETS, E.SCHED_SHARDED_FC, E.SCHED_SERIAL] + (
        [E.SCHED_FACTORS, E.SCHED_DEFER] if dtype == "fp32" else [])
    seq.append(E.SCHED_BUCKETS)
    outs = []
    for kind in ("eager", "shm"):
        eng = mnist_engine(di, "buckets", dtype, kind)
        for sch in seq:
            eng._set_schedule(sch)
            eng.train(G + 1)
        outs.append(finish(eng))
    same(outs[1], outs[0], "captured switching sequence vs eager")
    # the serial emulation of data parallelism (rank 0): buckets == serial
    if di.rank == 0:
        p1, m1 = NS.serial(dtype, STEPS, di.world)
        same(eager["buckets"], (p1, m1), "buckets vs serial emulation")
    return f"schedules={','.join(scheds)} tuned={picked}"


def scenario_xgmi(di, dtype):
    from mpi_tensorflow_amd.parallel.comm import XgmiDeviceComm

    xc = XgmiDeviceComm(di, timeout_s=20.0)
    # generic in-place all-reduce of a registered buffer (segments of unequal
    # length: 100,004 floats over 2 ranks) and the segment gather, vs gloo
    g = torch.Generator().manual_seed(11 + di.rank)
    host = torch.randn(100_004, generator=g)
    t = host.cuda()
    xc.register(t)
    want = host.clone()
    dist.all_reduce(want)
    for _ in range(3):  # repeated: the per-block epochs advance
        t.copy_(host.cuda())
        xc.all_reduce_(t)
        torch.cuda.synchronize()
        assert torch.equal(t.cpu(), want), "xgmi all-reduce != gloo sum"
    t.copy_(host.cuda())
    xc._c.gather_segments(ptr(t), t.numel(), stream_handle())
    torch.cuda.synchronize()
    seg = (t.numel() // 4 + di.world - 1) // di.world * 4
    parts = [torch.empty_like(host) for _ in range(di.world)]
    dist.all_gather(parts, host)
    for r in range(di.world):
        lo, hi = r * seg, min(t.numel(), (r + 1) * seg)
        assert torch.equal(t.cpu()[lo:hi], parts[r][lo:hi]), f"gather: segment {r}"
    assert xc.error() == 0, "an xgmi barrier timed out"
    # the MNIST schedules over the xgmi communicator vs the eager buckets run
    # (xgmi-fac, fp32: vs the eager factor schedule - the same FC gradients
    # from the same gathered rows, another summation order than buckets)
    ref, _ = run_fixed(di, "buckets", dtype, "eager")
    refs = {"buckets": ref}
    scheds = ["xgmi", "serial"]
    if dtype == "fp32":
        refs["factors"], _ = run_fixed(di, "factors", dtype, "eager")
        scheds += ["xgmi-step", "xgmi-fac"]
    picked = []
    for sched in scheds + ["auto"]:
        cfg = C.TrainConfig(sync_schedule=sched, dtype=dtype, graph=True, graph_steps=G).validate()
        x, y = NS._shard(di.rank, di.world, cfg.seed)
        comm = XgmiDeviceComm(di, timeout_s=20.0)
        eng = NativeMnistEngine(cfg, x, y, torch.device("cuda"), di.rank, di.world, comm)
        assert eng.use_graph and eng.xcomm is comm
        if sched != "auto":
            assert eng.sync_schedule == sched, (eng.sync_schedule, sched)
        eng.train(STEPS)
        assert comm.error() == 0, f"{sched}: an xgmi barrier timed out"
        got = eng.sync_schedule
        want = refs["factors"] if got == "xgmi-fac" else ref
        same(finish(eng), want, f"xgmi comm, {got} (captured) vs eager "
             + ("factors" if got == "xgmi-fac" else "buckets"))
        picked.append(got)
    return f"all_reduce+gather ok; schedules {','.join(scheds)}, auto->{picked[-1]}"


def scenario_xgmi_gate(di):
    """the exactness gate and the trial-step compare."""
    from mpi_tensorflow_amd.parallel.comm import (XgmiDeviceComm, exact_pattern, exact_sum,
                                                  xgmi_exactness_check)

    cfg = C.TrainConfig(graph=True, graph_steps=G).validate()
    shm = ShmDeviceComm(di, comm_capacity_bytes(cfg), timeout_s=60.0)
    good = XgmiDeviceComm(di, timeout_s=20.0)
    assert xgmi_exactness_check(good, shm) is None, "a healthy communicator failed the gate"
    # the fault on both ranks: identical on both ranks, and wrong
    bad = XgmiDeviceComm(di, timeout_s=20.0)
    bad.inject_skip_peer(1)
    t = exact_pattern(di.rank, 9, 1 << 20).cuda()
    bad.register(t)
    bad.all_reduce_(t)
    torch.cuda.synchronize()
    assert replicas_identical(t), "the skip-peer fault should leave the replicas identical"
    assert not torch.equal(t.cpu(), exact_sum(di.world, 9, 1 << 20)), "the fault did not bite"
    why = xgmi_exactness_check(bad, shm)
    assert why is not None and "exact integer sum" in why, why
    assert bad.error() == 0
    # the MNIST auto-tune: xGMI candidates next to the shm schedules
    picks = {}
    for fault in (False, True):
        x, y = NS._shard(di.rank, di.world, cfg.seed)
        xc = XgmiDeviceComm(di, timeout_s=20.0)
        assert xgmi_exactness_check(xc, shm) is None
        comm = ShmDeviceComm(di, comm_capacity_bytes(cfg), timeout_s=60.0)
        eng = NativeMnistEngine(cfg, x, y, torch.device("cuda"), di.rank, di.world, comm, xcomm=xc)
        if fault:
            xc.inject_skip_peer(1)
        p0 = eng.params.clone()
        eng.tune_schedule()
        assert torch.equal(eng.params, p0), "tune changed the state"
        xg = [k for k in eng.tune_log if k.startswith("xgmi")]
        assert xg, eng.tune_log
        if fault:
            assert all(eng.tune_log[k] is None for k in xg), eng.tune_log
            assert all("trial step differs" in eng.tune_reject[k] for k in xg), eng.tune_reject
            assert not eng.sync_schedule.startswith("xgmi")
        else:
            assert all(eng.tune_log[k] is not None for k in xg), (eng.tune_log, eng.tune_reject)
            assert eng.xgmi_step_check and max(eng.xgmi_step_check.values()) < 1e-4
        picks[fault] = eng.sync_schedule
        eng.train(STEPS)
        finish(eng)
    return f"gate ok; picks {picks}"


def scenario_param_avg(di):
    outs = {}
    for kind in ("shm",):
        eng = mnist_engine(di, "auto", "fp32", kind, sync="param_avg")
        assert not eng.grad_sync
        comm = eng.comm
        eng.train(4)
        torch.cuda.synchronize()
        mine = eng.params.cpu()
        parts = [torch.empty_like(mine) for _ in range(di.world)]
        dist.all_gather(parts, mine)
        average_params(comm, eng.params)
        torch.cuda.synchronize()
        want = parts[0].clone()
        for p in parts[1:]:
            want += p
        want *= 1.0 / di.world
        assert torch.equal(eng.params.cpu(), want), "param_avg != mean of the replicas"
        assert replicas_identical(eng.params)
        # root-only quirk (Q11): rank 0 gets the mean of the four weight
        # tensors, biases and every other rank are untouched
        eng.train(3)
        torch.cuda.synchronize()
        mine = eng.params.cpu()
        parts = [torch.empty_like(mine) for _ in range(di.world)]
        dist.all_gather(parts, mine)
        average_params_root_only(comm, eng.layout, eng.params)
        torch.cuda.synchronize()
        got = eng.layout.views(eng.params.cpu())
        mv = eng.layout.views(mine)
        for s in eng.layout.specs:
            if di.rank == 0 and s.name in REFERENCE_AVERAGED:
                w = sum(eng.layout.views(p)[s.name] for p in parts) / di.world
                assert torch.equal(got[s.name], w), f"root-only: {s.name} is not the mean"
            else:
                assert torch.equal(got[s.name], mv[s.name]), f"root-only touched {s.name}"
        outs[kind] = True
    return "all-ranks + root-only"


def scenario_generic(di, model):
    from mpi_tensorflow_amd.models.generic import model_input_shape
    from mpi_tensorflow_amd.runtime.generic_engine import GenericEngine
    from mpi_tensorflow_amd.runtime.lenet_engine import NativeLenetEngine
    from mpi_tensorflow_amd.utils.data import synthetic_images_torch

    # LeNet-5 over xGMI: -xgmipush = the push sync in the update launch,
    # -xgmipull = the one-shot pull of every rank's double-buffered gradient
    xmode = "two-phase"
    for m in ("push", "pull"):
        if model.endswith("-xgmi" + m):
            xmode, model = m, model[:-4]
    xg = model.endswith("-xgmi")  # the xGMI peer-to-peer communicator instead of shm
    model = model[:-5] if xg else model
    fused = model == "lenet5-native"
    name = "lenet5" if fused else model
    Eng = NativeLenetEngine if fused else GenericEngine
    B = 64 if name == "lenet5" else 4
    steps = 7 if fused else 5  # resnet: 3 eager warm-up steps + one 2-step graph
    rows = 4 * B
    cfg = C.TrainConfig(model=name, batch_size=B, graph=True, graph_steps=2,
                        xgmi_mode=xmode).validate()

    def shard(r):
        x, y = synthetic_images_torch(rows, model_input_shape(name), seed=cfg.seed, start=r * rows)
        return x.numpy(), y.numpy()

    dev = torch.device("cuda")
    if xg:
        from mpi_tensorflow_amd.parallel.comm import XgmiDeviceComm
        comm = XgmiDeviceComm(di, timeout_s=20.0)
    else:
        comm = ShmDeviceComm(di, comm_capacity_bytes(cfg), timeout_s=60.0)
    eng = Eng(cfg, *shard(di.rank), dev, di.rank, di.world, comm)
    assert eng.grad_sync and eng.use_graph
    eng.train(steps)
    torch.cuda.synchronize()
    assert eng.use_graph and len(eng._graphs) >= 1, "the step was not captured"
    eng.sync_optimizer_state()
    p = eng.params.detach().cpu()
    assert replicas_identical(eng.params.detach()), "replicas diverged"
    if xg:
        assert comm.error() == 0, "an xgmi barrier timed out"
        assert replicas_identical(eng.mom.detach()), "momentum replicas diverged"
    if di.rank == 0:
        ecfg = C.TrainConfig(model=name, batch_size=B, graph=False).validate()
        engs = [Eng(ecfg, *shard(r), dev, r, di.world, None) for r in range(di.world)]
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
            for e in engs[1:]:
                lead.grads.add_(e.grads)
            if fused:
                native().optim.sgd_momentum(ptr(lead.params), ptr(lead.grads), ptr(lead.mom),
                                            lead.layout.total, 0, 0.0, cfg.momentum,
                                            1.0 / di.world, ptr(lead.lr_dev), 0.0,
                                            ptr(lead.step_dev), stream_handle())
            else:
                lead.update_gpu(1.0 / di.world)
        torch.cuda.synchronize()
        q = lead.params.detach().cpu()
        assert torch.equal(p, q), f"captured {model} vs serial emulation: {(p - q).abs().max().item()}"
        if xg:
            mq = lead.mom.detach().cpu()
            assert torch.equal(eng.mom.detach().cpu(), mq), "xgmi momentum vs serial emulation"
        assert np.isfinite(p.numpy()).all()
    if fused and xg:
        assert eng.xgmi_mode == xmode
    return f"model={model}{'-xgmi' if xg else ''} mode={xmode} steps={steps}"


def main():
    di = D.init("cuda")
    scen = sys.argv[1]
    arg = sys.argv[2] if len(sys.argv) > 2 else ""
    if scen == "mnist":
        msg = scenario_mnist(di, arg or "fp32")
    elif scen == "xgmi":
        msg = scenario_xgmi(di, arg or "fp32")
    elif scen == "xgmi_gate":
        msg = scenario_xgmi_gate(di)
    elif scen == "param_avg":
        msg = scenario_param_avg(di)
    elif scen == "generic":
        msg = scenario_generic(di, arg)
    else:
        raise SystemExit(f"unknown scenario {scen}")
    D.barrier()
    if di.rank == 0:
        print(f"CAPTURED_SYNC_OK {scen} {arg} world={di.world} {msg}", flush=True)
    D.shutdown()


if __name__ == "__main__":
    main()
