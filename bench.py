"""Headline benchmark: MNIST CNN training throughput, images/sec (whole node).

Config = the reference workload: the 2-layer MNIST CNN of
/root/reference/mpipy.py:155-167, per-rank batch 64, momentum SGD with the
reference LR schedule, fp32 compute, synthetic MNIST-shaped data and random
init, data parallel over N GPUs with a per-step gradient all-reduce (RCCL
over xGMI, overlapped with backward).  Weak scaling: global batch = 64 * N.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

Without a launcher, `--gpus N` (N > 1) starts the N rank processes itself
(one per GPU, LOCAL_RANK = GPU index, rendezvous on 127.0.0.1) before this
process touches the GPU, relays their output and exits non-zero if any rank
fails; a rank whose world size differs from --gpus exits non-zero too.

Each rank runs W untimed steps, then EXACTLY K timed steps bracketed by a
barrier + device synchronize on both sides; the slowest rank's time is
used; rank 0 prints one JSON line.  Every timed step is a full training
step (forward, backward, all-reduce, SGD update); eval is outside the
timed region.  Before the W warm-up steps, --prewarm-ms (default 1000) of
forward-only test-set passes bring the GPU out of its idle clock state (no
training state changes; reported as prewarm / prewarm_ms).  --prewarm train
replays the captured training graph instead, on snapshotted state that is
restored afterwards: a second of it at full load leaves the clocks lower
for the short timed window that follows (20 steps: 125-133 us vs 85-92
after the eval passes on one box, final round-4 build; steady state 84).  With N > 1 the
sync schedule is autotuned first (real training steps, reported), and
after the run every rank's weights are checksummed: replicas that differ
fail the run (replicas_identical in the JSON).
"""

from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import torch

METRIC = "images/sec (whole node) + final test accuracy, MNIST CNN at 1/2/4/8 MI355X"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--model", default="mnist_cnn", choices=("mnist_cnn", "lenet5", "resnet18"))
    ap.add_argument("--batch-size", type=int, default=None,
                    help="per-GPU batch (default 64; 32 for resnet18)")
    ap.add_argument("--dtype", default="fp32", choices=("fp32", "bf16"))
    ap.add_argument("--sync", default="grad", choices=("grad", "none"))
    ap.add_argument("--graph-steps", type=int, default=25)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--backend", default="auto", choices=("auto", "native", "torch"))
    ap.add_argument("--no-eval", action="store_true")
    ap.add_argument("--sync-schedule", default="auto",
                    choices=("auto", "buckets", "sharded", "split", "factors", "serial", "defer",
                             "xgmi", "xgmi-step", "xgmi-fac"))
    ap.add_argument("--defer-split", type=float, default=0.5,
                    help="defer schedule: fraction of the FC bucket reduced under the conv backward")
    ap.add_argument("--comm", default="auto", choices=("auto", "rccl", "shm", "xgmi", "torch"),
                    help="device communicator (auto: RCCL, or shared memory when ranks share "
                         "GPUs; on one node the xGMI peer-to-peer schedule is also tuned)")
    ap.add_argument("--no-xgmi", action="store_true",
                    help="comm auto: do not set up the xGMI peer-to-peer communicator")
    ap.add_argument("--bn-fused", choices=("on", "off"), default=None,
                    help="BatchNorm finalize fused into the apply launch (grid barrier) or "
                         "the separate finalize launch (A/B; default: the library's)")
    ap.add_argument("--bn-fused-bpc", type=int, default=None,
                    help="fused BatchNorm grid: blocks a CU (1..8)")
    ap.add_argument("--tiled-plan", default="",
                    help="generic conv TiledPlan overrides, k=v comma list (A/B labs; "
                         "e.g. vcap=128,halo_f32_bm=128)")
    ap.add_argument("--xgmi-mode", default="pull", choices=("two-phase", "push", "pull"),
                    help="lenet5 over xGMI: the two-phase all-reduce + SGD launch, the push sync "
                         "fused into the update launch, or the one-barrier pull of every rank's "
                         "double-buffered gradient (comm auto tunes all three)")
    ap.add_argument("--xgmi-push", action="store_true", help="= --xgmi-mode push")
    ap.add_argument("--xgmi-inject-skip-peer", type=int, default=-1, metavar="R",
                    help="failure injection (tests): the xGMI phase-1 reductions leave out rank "
                         "R; the exactness gate must then reject the xGMI communicator")
    ap.add_argument("--xgmi-emulate", default=None, metavar="LAT_US,LINK_GBPS[,N]",
                    help="1 GPU, MNIST: the xGMI peer-to-peer schedule against N (default 8) "
                         "virtual ranks whose phases last at least their bytes on one link at "
                         "LINK_GBPS per direction, plus LAT_US per barrier (timing only)")
    ap.add_argument("--grad-comm-dtype", default="fp32", choices=("fp32", "bf16"),
                    help="wire dtype of the gradient all-reduce (bf16: half the xGMI bytes)")
    ap.add_argument("--comm-emulate", default=None, metavar="LAT_US,BUSBW_GBPS[,N[,BLOCKS]]",
                    help="1 GPU: replace the collectives by timing stand-ins of an N-rank ring "
                         "(default N=8, 32 workgroups) to measure sync/compute overlap")
    ap.add_argument("--force-sync", action="store_true",
                    help="1 GPU: run the RCCL all-reduce path anyway (world-1 communicator), "
                         "to measure the overhead of the comm stream and buckets")
    ap.add_argument("--prewarm-ms", type=float, default=1000.0,
                    help="untimed forward-only test-set passes before the warm-up steps (no "
                         "training state changes) so a short timed window does not measure "
                         "the GPU clock ramp (1 GPU: 20 replayed steps ran 114.8 -> 109.6 us "
                         "over the first 120 steps, steady state 108.6)")
    ap.add_argument("--prewarm", default="eval", choices=("eval", "train"),
                    help="what the prewarm runs: forward-only test-set passes (eval), or "
                         "training-graph replays on snapshotted state that is restored "
                         "afterwards (train; engines with prewarm_train, else eval)")
    ap.add_argument("--bucket-plan", default="auto",
                    help="resnet18: gradient all-reduce buckets (auto: timed at start-up over "
                         "parallel/overlap.py BUCKET_PLANS / layout / one / bytes:MiB / geo:RATIO)")
    ap.add_argument("--bucket-mb", type=float, default=None,
                    help="resnet18: shorthand for --bucket-plan bytes:MiB")
    ap.add_argument("--collective-timeout-s", type=float, default=300.0,
                    help="watchdog deadline per device-waiting region (N > 1): a hung or "
                         "failed collective aborts the communicators and exits non-zero")
    return ap.parse_args(argv)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def gpu_count_sysfs() -> int:
    """GPUs visible to this process, counted from the KFD topology in sysfs
    (nodes with SIMDs) and the *_VISIBLE_DEVICES masks: no HIP call, so the
    spawning parent can never initialise the GPU runtime.  -1 if unknown."""
    import glob

    n = 0
    try:
        for f in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
            with open(f) as fh:
                for line in fh:
                    k, _, v = line.partition(" ")
                    if k == "simd_count" and int(v) > 0:
                        n += 1
    except (OSError, ValueError):
        return -1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip() != ""]))
    return n


def launch_ranks(n: int, argv, share_gpus: bool = False) -> int:
    """Starts n rank processes of this script (no torchrun / mpirun in the
    environment).  The parent makes no HIP call at all (GPUs are counted from
    sysfs), so the children are fresh processes, not re-execs.  Rank 0's
    stdout (the JSON line) is inherited; the first failing rank makes the
    parent stop the others and return its exit code."""
    ndev = gpu_count_sysfs()
    if 0 < ndev < n and not share_gpus:
        print(f"error: --gpus {n} but only {ndev} GPU(s) visible", file=sys.stderr)
        return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv),
                                      env=env))
    rc = 0
    live = list(range(n))
    while live:
        for r in list(live):
            c = procs[r].poll()
            if c is None:
                continue
            live.remove(r)
            if c != 0 and rc == 0:
                rc = c
                print(f"error: rank {r} exited with {c}; stopping the other ranks", file=sys.stderr)
                for o in live:
                    procs[o].terminate()
        time.sleep(0.05)
    for p in procs:
        p.wait()
    return rc


def prewarm(eng, x, y, ms: float) -> float:
    """Forward-only eval passes over (a slice of) the test set until `ms` of
    wall time has passed: the GPU leaves its idle clock state before the
    warm-up steps.  Weights, momentum, step counter and data order are
    untouched (evaluate() runs the inference kernels only)."""
    if ms <= 0:
        return 0.0
    n = min(2000, int(x.shape[0]))
    xs, ys = x[:n], y[:n]  # one object: engines that keep the eval set resident upload it once
    t0 = time.perf_counter()
    while 1000.0 * (time.perf_counter() - t0) < ms:
        eng.evaluate(xs, ys)
    return round(1000.0 * (time.perf_counter() - t0), 1)


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else list(argv)
    a = parse(argv)
    from mpi_tensorflow_amd.parallel import dist as D
    from mpi_tensorflow_amd.parallel.watchdog import make_watchdog
    from mpi_tensorflow_amd.utils.faults import maybe_fail

    if a.gpus > 1 and D.discover().launcher == "none":
        # --comm shm / auto / xgmi: ranks may share GPUs (rank r binds GPU r %
        # count; auto then picks the shared-memory communicator, parallel/comm.py;
        # xgmi maps the other ranks' buffers on the same device)
        return launch_ranks(a.gpus, argv, share_gpus=a.comm in ("shm", "auto", "xgmi"))
    if D.discover().world != a.gpus:
        print(f"error: --gpus {a.gpus} but the launcher started {D.discover().world} rank(s)",
              file=sys.stderr)
        return 2
    device = D.resolve_device("auto")
    di = D.init(str(device))
    N = di.world
    if device.type == "cuda" and (a.bn_fused is not None or a.bn_fused_bpc is not None
                                  or a.tiled_plan):
        from mpi_tensorflow_amd.ops import native as _native
        if a.tiled_plan:
            plan = _native().ops.get_tiled_plan()
            for kv in a.tiled_plan.split(","):
                k, v = kv.split("=")
                cur = getattr(plan, k)
                setattr(plan, k, (v not in ("0", "false")) if isinstance(cur, bool) else int(v))
            _native().ops.set_tiled_plan(plan)
        if a.bn_fused is not None:
            _native().ops.bn_set_fused(a.bn_fused == "on")
        if a.bn_fused_bpc is not None:
            _native().ops.bn_set_fused_blocks_per_cu(a.bn_fused_bpc)
    maybe_fail("after_init", di.rank)
    # the watchdog exists before the communicator: start-up collectives
    # (communicator init, the engines' connection setup) are guarded too
    wd = make_watchdog([], a.collective_timeout_s, di.rank, N)
    try:
        return run(a, di, device, wd)
    finally:
        wd.stop()


def run(a, di, device, wd) -> int:
    from mpi_tensorflow_amd import config as C
    from mpi_tensorflow_amd.parallel import dist as D
    from mpi_tensorflow_amd.parallel.setup import check_health, setup_comms
    from mpi_tensorflow_amd.parallel.watchdog import run_in_chunks
    from mpi_tensorflow_amd.runtime.mnist_engine import make_engine
    from mpi_tensorflow_amd.utils.data import load_mnist_shard
    from mpi_tensorflow_amd.utils.faults import maybe_fail

    N = di.world
    if a.batch_size is None:
        a.batch_size = 32 if a.model == "resnet18" else 64
    cfg = C.TrainConfig(model=a.model, batch_size=a.batch_size, dtype=a.dtype, sync=a.sync,
                        graph=not a.no_graph, graph_steps=a.graph_steps, backend=a.backend,
                        sync_schedule=a.sync_schedule, comm=a.comm,
                        defer_split=a.defer_split, grad_comm_dtype=a.grad_comm_dtype,
                        bucket_plan=f"bytes:{a.bucket_mb:g}" if a.bucket_mb else a.bucket_plan,
                        collective_timeout_s=a.collective_timeout_s,
                        no_xgmi=a.no_xgmi,
                        xgmi_mode="push" if a.xgmi_push else a.xgmi_mode).validate()
    force = bool((a.force_sync or a.comm_emulate or a.xgmi_emulate) and N == 1
                 and device.type == "cuda")
    with wd.guard("start-up (communicator, engine)"):
        maybe_fail("before_comm", di.rank)
        # the same set-up as the mpipy.py Trainer (parallel/setup.py): the device
        # comm and, on one node, the exactness-gated xGMI candidate
        if a.xgmi_inject_skip_peer >= 0:
            import mpi_tensorflow_amd.parallel.comm as CM
            CM.INJECT_SKIP_PEER = a.xgmi_inject_skip_peer
        comms = setup_comms(di, device, cfg, no_xgmi=a.no_xgmi,
                            xgmi_timeout_s=min(20.0, a.collective_timeout_s))
        comm, xcomm = comms.comm, comms.xcomm
        if force and a.xgmi_emulate:
            from mpi_tensorflow_amd.parallel.comm import XgmiDeviceComm, xgmi_exactness_check
            f = [float(v) for v in a.xgmi_emulate.split(",")]
            xe = XgmiDeviceComm.emulated(int(f[2]) if len(f) > 2 else 8, f[0], f[1])
            if a.xgmi_inject_skip_peer >= 0:
                xe.inject_skip_peer(a.xgmi_inject_skip_peer)
            why = xgmi_exactness_check(xe)
            comms.xgmi_status = "passed" if why is None else f"dropped: exactness check failed ({why})"
            if why is not None:
                print(f"error: the emulated xGMI communicator failed its exactness check ({why})",
                      file=sys.stderr)
                return 5
            if a.comm_emulate:  # both: the xGMI schedule is a candidate next to the RCCL ones
                xcomm = xe
            else:
                comm = xe
        if force and a.comm_emulate:
            from mpi_tensorflow_amd.parallel.comm import EmulatedDeviceComm
            f = [float(v) for v in a.comm_emulate.split(",")]
            comm = EmulatedDeviceComm(int(f[2]) if len(f) > 2 else 8, f[0], f[1],
                                      int(f[3]) if len(f) > 3 else 32)
        elif force and not a.xgmi_emulate:
            from mpi_tensorflow_amd.parallel.comm import RcclDeviceComm
            comm = RcclDeviceComm(di)
        wd.add(comm)
        maybe_fail("after_comm", di.rank)
        if a.model == "mnist_cnn":
            shard = load_mnist_shard(di.rank, N, synthetic=True, seed=cfg.seed)
            eng = make_engine(cfg, shard.train_x, shard.train_y, device, di.rank, N, comm,
                              force_sync=force, xcomm=xcomm)
            test_x, test_y = shard.test_x, shard.test_y
        else:
            from mpi_tensorflow_amd.models.generic import model_input_shape
            from mpi_tensorflow_amd.runtime.generic_engine import make_image_engine
            from mpi_tensorflow_amd.utils.data import synthetic_images_torch

            shape = model_input_shape(a.model)
            if a.model == "lenet5":  # the Trainer's task (utils/data.py v2 design)
                from mpi_tensorflow_amd.utils.data import synthetic_image_shard

                sh = synthetic_image_shard(di.rank, N, 8192, 2048, shape, seed=cfg.seed)
                tx, ty, test_x, test_y = sh.train_x, sh.train_y, sh.test_x, sh.test_y
            else:
                rows = max(4 * a.batch_size, 256)
                txt, tyt = synthetic_images_torch(rows, shape, seed=cfg.seed, start=di.rank * rows)
                ext, eyt = synthetic_images_torch(256, shape, seed=cfg.seed, split="test",
                                                  start=di.rank * 256)
                tx, ty, test_x, test_y = txt.numpy(), tyt.numpy(), ext.numpy(), eyt.numpy()
            eng = make_image_engine(cfg, tx, ty, device, di.rank, N, comm, force_sync=force,
                                    xcomm=xcomm)
        wd.add(getattr(eng, "comm2", None))

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize()

    # startup autotune of the gradient-sync schedule (N > 1, native MNIST
    # engine): trial steps that are discarded (params / momentum / step are
    # restored), before the warm-up, outside the timing
    with wd.guard("sync-schedule autotune and capture"):
        tune_steps = eng.tune_schedule() if hasattr(eng, "tune_schedule") else 0
        if hasattr(eng, "capture"):
            eng.capture(a.warmup)
            eng.capture(a.steps)
        pw_ms = a.prewarm_ms if device.type == "cuda" else 0.0
        prewarm_mode = "train" if a.prewarm == "train" and hasattr(eng, "prewarm_train") else "eval"
        if prewarm_mode == "train":
            prewarm_ms = eng.prewarm_train(pw_ms)
        else:
            prewarm_ms = prewarm(eng, test_x, test_y, pw_ms)
        sync()
    maybe_fail("before_train", di.rank)
    chunks = {}
    run_in_chunks(wd, eng.train, sync, a.warmup, "warm-up steps",
                  granule=getattr(eng, "graph_steps", 1), state=chunks)
    D.barrier()
    sync()
    with wd.guard(f"timed steps ({a.steps})"):  # arming is two attribute writes
        t0 = time.perf_counter()
        eng.train(a.steps)
        sync()
        t1 = time.perf_counter()
    D.barrier()
    dt = D.allreduce_max_host(t1 - t0)
    if N > 1:  # every rank stops when any rank's xGMI barrier timed out
        check_health("timed steps", comm, eng)
    err = float("nan")
    if not a.no_eval:
        # accuracy of the reference's full run: MNIST trains `epochs` local
        # epochs (mpipy.py:79, 2 x N_local // 64 steps per rank); the timed
        # steps count towards it and the rest run untimed here (fast: the
        # same captured graphs).  The other models stop at warmup + steps.
        if a.model == "mnist_cnn":
            from mpi_tensorflow_amd.utils.data import steps_per_run

            run_in_chunks(wd, eng.train, sync,
                          max(0, steps_per_run(eng.n_local, cfg.epochs, a.batch_size) - eng.step),
                          "accuracy-run steps", first_step=eng.step,
                          granule=getattr(eng, "graph_steps", 1), state=chunks)
        err = D.allreduce_sum_host(eng.evaluate(test_x, test_y)) / N
    # replica consistency (N > 1, per-step gradient sync): every rank must hold
    # bit-identical weights after the run; a mismatch means a lost or corrupted
    # collective, and the run fails loudly (outside the timing)
    replicas = None
    if N > 1 and a.sync == "grad" and getattr(eng, "params", None) is not None:
        from mpi_tensorflow_amd.parallel.sync import replicas_identical

        if hasattr(eng, "sync_optimizer_state"):
            eng.sync_optimizer_state()
        sync()
        replicas = replicas_identical(eng.params) and replicas_identical(eng.mom)
    images = N * a.batch_size * a.steps
    value = images / dt
    if a.model == "mnist_cnn":
        model_desc = "mnist_cnn (2-layer MNIST CNN of mpipy.py: conv5x5x32-pool-conv5x5x64-pool-fc512-dropout-fc10)"
        image, data_desc = "28x28x1", "synthetic (MNIST-shaped 28x28x1, class-conditional; random-init weights)"
    elif a.model == "lenet5":
        model_desc = "lenet5 (conv5x5x6-pool-conv5x5x16-pool-fc120-fc84-fc10)"
        image, data_desc = "32x32x3", "synthetic (CIFAR-shaped 32x32x3, shared-template task v2; random-init weights)"
    else:
        model_desc = "resnet18 (BasicBlock [2,2,2,2], BatchNorm, 10 classes)"
        image, data_desc = "224x224x3", "synthetic (ImageNet-shaped 224x224x3, shared-template task v2; random-init weights)"
    # as the library reports it (an emulated communicator stands in for more ranks)
    comm_nranks = comm.nranks if hasattr(comm, "nranks") and not force else None
    if comm_nranks is not None and comm_nranks != N:
        print(f"error: the communicator has {comm_nranks} ranks, expected {N}", file=sys.stderr)
        return 3
    if di.rank == 0:
        out = {
            "metric": METRIC if a.model == "mnist_cnn" else f"images/sec (whole node), {a.model}",
            "value": round(value, 1),
            "unit": "images/sec",
            "n_gpus": N,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1000.0 * dt / a.steps, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": getattr(getattr(eng, "cfg", None), "dtype", a.dtype),  # effective
            "data": data_desc,
            "config": {
                "model": model_desc,
                "global_batch": a.batch_size * N,
                "per_gpu_batch": a.batch_size,
                "seq_len": None,
                "image": image,
                "parallelism": f"dp{N}",
                "sync": ("per-step gradient all-reduce" if (N > 1 or force)
                         else "none (1 rank)"),
                "engine": eng.kind,
                "comm": getattr(comm, "kind", "none"),
                "xgmi_comm": getattr(xcomm, "kind", None),
                "xgmi_gate": comms.xgmi_status,
                "ranks": N,
                "comm_nranks": comm_nranks,
                "sync_schedule": getattr(eng, "sync_schedule", "n/a"),
                "grad_comm_dtype": a.grad_comm_dtype,
                "sync_tune_us_per_step": getattr(eng, "tune_log", {}) or None,
                "sync_tune_steps": tune_steps,
                "graph_steps": (a.graph_steps if not a.no_graph else 0),
                "prewarm_ms": prewarm_ms,
                "prewarm": prewarm_mode,
                "replicas_identical": replicas,
                # generic engines' segmented step: nodes of each overlapped
                # bucket's collective graph (N > 1: every one moves bytes)
                "collective_graph_nodes": (eng.collective_graph_nodes()
                                           if hasattr(eng, "collective_graph_nodes") else None),
            },
            "final_test_accuracy": None if err != err else round(100.0 - err, 3),
            "test_eval_after_steps": int(eng.step),
            "test_rows": int(test_x.shape[0]) * N,
        }
        print(json.dumps(out))
        sys.stdout.flush()
    D.barrier()
    D.shutdown()
    if replicas is False:
        print("error: the ranks' weights differ after the run (replica checksum mismatch)",
              file=sys.stderr)
        return 4
    return 0


if __name__ == "__main__":
    sys.exit(main())
