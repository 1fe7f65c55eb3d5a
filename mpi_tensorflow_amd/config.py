"""Global configuration: the reference's hard-coded constants plus CLI overrides.

The reference keeps every knob as a module global or an inline literal
(`/root/reference/mpipy.py:14-21` globals, `:57` L2 coefficient, `:60-64`
learning-rate schedule, `:65` momentum, `:87` sync period, `:166` dropout).
This module mirrors those defaults exactly and exposes them through one
dataclass (`TrainConfig`) plus an argparse builder, so the one-script API
(`mpipy.py`) keeps the reference defaults while every value is overridable.

`--reference-quirks` re-enables the reference's behavioural oddities that
the framework fixes by default:
  * Q5  - train shard padded with zero rows (tr_size//P rows, 5000/P zeros)
  * Q8  - dropout stays active at evaluation time
  * Q9  - full local test-set evaluation after every training step
  * Q11 - "bcast" = gather weights (not biases/momentum) to rank 0 and
          average there only; other ranks never receive the average
  * Q14 - identical dropout seeds on every rank
"""

from __future__ import annotations

import argparse
import dataclasses
import os
from typing import List, Optional

# --- reference constants (mpipy.py:14-21) -------------------------------
# mpipy.py:14 sets TF_CPP_MIN_LOG_LEVEL=2 and :15 MPI_OPTIMAL_PATH=1; the
# equivalents here are log verbosity knobs, not environment variables.
DATA_URL = "https://storage.googleapis.com/cvdf-datasets/mnist/"  # mpipy.py:17
ITERATION = 2  # epochs over the local shard, mpipy.py:18
IMAGE_SIZE = 28  # mpipy.py:19
BATCH_SIZE = 64  # per-rank batch, mpipy.py:20
NUM_CHANNEL = 10  # number of classes (named "channel" in mpipy.py:21)
NUM_CLASSES = NUM_CHANNEL
PIXEL_DEPTH = 255.0  # tutorial extract_data scaling: (x - 127.5) / 255

# --- optimisation constants (mpipy.py:57-66) ------------------------------
BASE_LR = 0.01  # mpipy.py:60
LR_DECAY = 0.95  # mpipy.py:63
MOMENTUM = 0.9  # mpipy.py:65
L2_COEF = 5e-4  # mpipy.py:57
DROPOUT_KEEP = 0.5  # mpipy.py:166
SEED = 1  # op seed of every truncated_normal and the dropout, mpipy.py:40,166
INIT_STDDEV = 0.1  # mpipy.py:39

# --- distributed constants ----------------------------------------------------
SYNC_EVERY = 50  # mpipy.py:87 (step>0 and step%50==0)
TRAIN_ROWS = 55000  # mpipy.py:211 (tr_size before rounding)
TEST_ROWS = 10000  # mpipy.py:212
VAL_ROWS = 5000  # mpipy.py:213
TRAIN_FILE_ROWS = 60000  # mpipy.py:216 (extract 60000 train images)

MNIST_FILES = {
    "train_images": "train-images-idx3-ubyte.gz",  # mpipy.py:203
    "train_labels": "train-labels-idx1-ubyte.gz",  # mpipy.py:204
    "test_images": "t10k-images-idx3-ubyte.gz",  # mpipy.py:205
    "test_labels": "t10k-labels-idx1-ubyte.gz",  # mpipy.py:206
}

MODELS = ("mnist_cnn", "lenet5", "resnet18")
SYNC_MODES = ("grad", "param_avg", "none")
# gradient-sync schedules of the native MNIST executor (grad sync, world > 1):
# "buckets" = all-reduce FC bucket then conv bucket; "sharded" = reduce-scatter
# FC grads + 1/N-shard SGD + all-gather overlapped with the next forward
# "split" = FC all-reduce + SGD on the comm stream, conv all-reduce on the
# compute stream over a second communicator
# "xgmi" = the peer-to-peer xGMI communicator's fused sync + SGD launch (MNIST,
# csrc/xgmi_comm.h; one node)
SYNC_SCHEDULES = ("auto", "buckets", "sharded", "split", "factors", "serial", "defer", "xgmi",
                  "xgmi-step", "xgmi-fac")
# device communicator (world > 1): "auto" = native RCCL when every rank has a
# GPU of its own, the shared-memory host-staged communicator when ranks share
# GPUs (the reference's layout: every rank on /GPU:0, quirk Q13); "rccl",
# "shm" and "torch" (torch.distributed) force one
# "xgmi": collectives as compute-stream kernels reading the peers' memory
# over the xGMI mesh (IPC-mapped; one node)
COMMS = ("auto", "rccl", "shm", "xgmi", "torch")
# LeNet-5's sync over the xGMI communicator (TrainConfig.xgmi_mode)
XGMI_MODES = ("two-phase", "push", "pull")
DTYPES = ("fp32", "bf16")


@dataclasses.dataclass
class TrainConfig:
    """Every knob of a training run.  Defaults = the reference's behaviour
    with its bugs fixed (see module docstring for the quirk switch)."""

    model: str = "mnist_cnn"
    epochs: int = ITERATION
    batch_size: int = BATCH_SIZE
    dtype: str = "fp32"
    # gradient all-reduce every step (default, arXiv:1603.02339 intent) or the
    # reference's periodic weight averaging (mpipy.py:87-91)
    sync: str = "grad"
    sync_every: int = SYNC_EVERY
    sync_schedule: str = "auto"
    # "defer" schedule: fraction of the FC bucket all-reduced under the conv
    # backward (the rest overlaps the next step's conv forward)
    defer_split: float = 0.5
    # dtype of the gradient collectives: fp32 (the reference's MPI Gather of
    # fp32 tensors) or bf16 (half the bytes over xGMI; the sum is rounded to
    # bf16 on the wire, the update stays fp32)
    grad_comm_dtype: str = "fp32"
    # generic models (ResNet-18): how the flat gradients are cut into
    # all-reduce buckets (parallel/overlap.py plan_layout); "auto" times the
    # BUCKET_PLANS candidates on the real communicator at startup
    bucket_plan: str = "auto"
    comm: str = "auto"
    # comm auto, one node: do not set up the xGMI peer-to-peer communicator as
    # an extra sync-schedule candidate (parallel/setup.py setup_comms)
    no_xgmi: bool = False
    # LeNet-5 over the xGMI communicator (--comm xgmi): "two-phase" (this
    # rank's segment summed + SGD, then the others gathered; sharded momentum),
    # "push" (the gradient pushed into the peers' receive slots from the update
    # launch, one barrier, kernels/lenet.h PushArgs) or "pull" (double-buffered
    # gradient slots, one launch reads every rank's whole gradient, one
    # barrier, replicated SGD; kernels/xgmi.h OneShotArgs); with --comm auto
    # all three are tuned next to RCCL.  Default pull: emulated 8 ranks at
    # 1 us / 150 GB/s 34.97 us a step against 42.31 two-phase, 44.1 push
    xgmi_mode: str = "pull"
    # fp32 MNIST conv2 algorithm on the native engine: "winograd" (F(2x2,5x5),
    # kernels/wino.h; 2.8x fewer MFMAs, fp32 arithmetic throughout, ~1e-6
    # relative error) or "direct" (25-tap implicit GEMM)
    conv_algo: str = "winograd"
    # restrict sync_schedule="auto" to the schedules whose updates are bit
    # identical to the bucketed all-reduce (the factor schedule sums the FC
    # gradients in another order, so an auto run that picked it is only
    # reproducible by naming it; the chosen schedule is logged either way)
    deterministic: bool = False
    # evaluate (and print the reference log line) every N steps; the
    # reference evaluates every step (Q9) but prints every 50
    eval_every: int = SYNC_EVERY
    # data
    data_dir: str = "data"
    synthetic: Optional[bool] = None  # None = use real files if present
    download: bool = False
    # learning rate / optimiser
    base_lr: float = BASE_LR
    lr_decay: float = LR_DECAY
    momentum: float = MOMENTUM
    l2: float = L2_COEF
    dropout_keep: float = DROPOUT_KEEP
    seed: int = SEED
    # execution
    backend: str = "auto"  # auto | native (HIP kernels) | torch (oracle path)
    device: str = "auto"  # auto | cpu | cuda
    graph: bool = True  # capture the step into a HIP graph (native backend)
    graph_steps: int = 10  # training steps per captured graph replay
    max_steps: Optional[int] = None  # cap on steps (None = epochs-derived)
    # checkpoint / metrics
    ckpt: Optional[str] = None
    ckpt_every: int = 0
    resume: Optional[str] = None
    metrics_jsonl: Optional[str] = None
    quiet: bool = False
    # robustness: process-group / collective timeout (a dead rank turns into
    # an error instead of a hang) and a cross-replica consistency probe at
    # every eval event in grad-sync mode (replicas must stay identical)
    collective_timeout_s: float = 600.0
    check_replicas: bool = False
    # compat
    reference_quirks: bool = False

    def validate(self) -> "TrainConfig":
        if self.model not in MODELS:
            raise ValueError(f"unknown model {self.model!r}; choose from {MODELS}")
        if self.sync not in SYNC_MODES:
            raise ValueError(f"unknown sync {self.sync!r}; choose from {SYNC_MODES}")
        if self.xgmi_mode not in XGMI_MODES:
            raise ValueError(f"unknown xgmi mode {self.xgmi_mode!r}; choose from {XGMI_MODES}")
        if self.sync_schedule not in SYNC_SCHEDULES:
            raise ValueError(f"unknown sync schedule {self.sync_schedule!r}; "
                             f"choose from {SYNC_SCHEDULES}")
        if not 0.0 < self.defer_split < 1.0:
            raise ValueError(f"defer_split must be in (0, 1), got {self.defer_split}")
        if self.grad_comm_dtype not in ("fp32", "bf16"):
            raise ValueError(f"unknown grad comm dtype {self.grad_comm_dtype!r}")
        if self.bucket_plan != "auto":
            from .parallel.overlap import check_plan
            check_plan(self.bucket_plan)
        if self.conv_algo not in ("winograd", "direct"):
            raise ValueError(f"unknown conv algo {self.conv_algo!r}")
        if self.comm not in COMMS:
            raise ValueError(f"unknown comm {self.comm!r}; choose from {COMMS}")
        if self.dtype not in DTYPES:
            raise ValueError(f"unknown dtype {self.dtype!r}; choose from {DTYPES}")
        if self.backend not in ("auto", "native", "torch"):
            raise ValueError(f"unknown backend {self.backend!r}")
        if self.batch_size <= 0 or self.epochs <= 0:
            raise ValueError("batch_size and epochs must be positive")
        if self.sync_every <= 0 or self.eval_every < 0:
            raise ValueError("sync_every must be > 0 and eval_every >= 0")
        if not 0.0 < self.dropout_keep <= 1.0:
            raise ValueError("dropout_keep must be in (0, 1]")
        return self

    # quirk accessors ------------------------------------------------------
    @property
    def pad_train_shard(self) -> bool:  # Q5
        return self.reference_quirks

    @property
    def eval_dropout(self) -> bool:  # Q8
        return self.reference_quirks

    @property
    def root_only_average(self) -> bool:  # Q11
        return self.reference_quirks

    @property
    def same_seed_all_ranks(self) -> bool:  # Q14
        return self.reference_quirks

    def effective_eval_every(self) -> int:  # Q9
        return 1 if self.reference_quirks else self.eval_every


def build_arg_parser(prog: str = "mpipy.py") -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(
        prog=prog,
        description="MI355X-native data-parallel CNN trainer (reference-compatible "
        "one-script API of mpi-Tensorflow's mpipy.py).",
    )
    d = TrainConfig()
    p.add_argument("--model", default=d.model, choices=MODELS)
    p.add_argument("--epochs", type=int, default=d.epochs, help="local epochs (mpipy.py:18)")
    p.add_argument("--batch-size", type=int, default=d.batch_size)
    p.add_argument("--dtype", default=d.dtype, choices=DTYPES)
    p.add_argument("--sync", default=d.sync, choices=SYNC_MODES)
    p.add_argument("--sync-every", type=int, default=d.sync_every)
    p.add_argument("--sync-schedule", default=d.sync_schedule, choices=SYNC_SCHEDULES,
                   help="native MNIST grad-sync schedule (auto / buckets / sharded FC update / "
                        "factors: all-gather the FC gradient factors, fp32 / defer: FC part B "
                        "overlaps the next conv forward, fp32)")
    p.add_argument("--defer-split", type=float, default=d.defer_split,
                   help="defer schedule: fraction of the FC bucket reduced under the conv backward")
    p.add_argument("--grad-comm-dtype", default=d.grad_comm_dtype, choices=("fp32", "bf16"),
                   help="wire dtype of the gradient all-reduce (bf16 halves the xGMI bytes)")
    p.add_argument("--bucket-plan", default=d.bucket_plan,
                   help="generic models: gradient all-reduce buckets (auto / layout / one / "
                        "bytes:MiB / geo:RATIO)")
    p.add_argument("--comm", default=d.comm, choices=COMMS,
                   help="device communicator: RCCL over xGMI (one GPU per rank), shm (host-"
                        "staged shared memory, ranks may share a GPU), xgmi (peer-to-peer "
                        "kernels on the compute stream, one node) or torch.distributed")
    p.add_argument("--no-xgmi", action="store_true",
                   help="comm auto: do not set up the xGMI peer-to-peer communicator "
                        "(otherwise gated by an exactness check, then tuned next to RCCL)")
    p.add_argument("--conv-algo", default=d.conv_algo, choices=("winograd", "direct"),
                   help="fp32 MNIST conv2 algorithm of the native engine")
    p.add_argument("--deterministic", action="store_true",
                   help="sync-schedule auto-tune picks only bit-identical schedules")
    p.add_argument("--eval-every", type=int, default=d.eval_every,
                   help="0 disables periodic eval")
    p.add_argument("--data-dir", default=d.data_dir)
    g = p.add_mutually_exclusive_group()
    g.add_argument("--synthetic", dest="synthetic", action="store_true", default=None)
    g.add_argument("--real-data", dest="synthetic", action="store_false")
    p.add_argument("--download", action="store_true", help="try DATA_URL if files missing")
    p.add_argument("--base-lr", type=float, default=d.base_lr)
    p.add_argument("--lr-decay", type=float, default=d.lr_decay)
    p.add_argument("--momentum", type=float, default=d.momentum)
    p.add_argument("--l2", type=float, default=d.l2)
    p.add_argument("--dropout-keep", type=float, default=d.dropout_keep)
    p.add_argument("--seed", type=int, default=d.seed)
    p.add_argument("--backend", default=d.backend, choices=("auto", "native", "torch"))
    p.add_argument("--device", default=d.device)
    p.add_argument("--no-graph", dest="graph", action="store_false", default=True)
    p.add_argument("--graph-steps", type=int, default=d.graph_steps)
    p.add_argument("--max-steps", type=int, default=None)
    p.add_argument("--ckpt", default=None, help="checkpoint path written at the end")
    p.add_argument("--ckpt-every", type=int, default=0)
    p.add_argument("--resume", default=None)
    p.add_argument("--metrics-jsonl", default=None)
    p.add_argument("--quiet", action="store_true")
    p.add_argument("--collective-timeout-s", type=float, default=d.collective_timeout_s,
                   help="process-group / collective timeout (seconds)")
    p.add_argument("--check-replicas", action="store_true",
                   help="verify at every eval that all ranks hold identical weights (grad sync)")
    p.add_argument("--reference-quirks", action="store_true",
                   help="reproduce mpipy.py quirks Q5/Q8/Q9/Q11/Q14")
    return p


def config_from_args(argv: Optional[List[str]] = None, prog: str = "mpipy.py") -> TrainConfig:
    ns = build_arg_parser(prog).parse_args(argv)
    kw = {f.name: getattr(ns, f.name) for f in dataclasses.fields(TrainConfig) if hasattr(ns, f.name)}
    return TrainConfig(**kw).validate()


def env_flag(name: str, default: bool = False) -> bool:
    v = os.environ.get(name)
    if v is None:
        return default
    return v.strip().lower() not in ("", "0", "false", "no", "off")
