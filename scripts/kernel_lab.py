"""Times every kernel of the native MNIST step in isolation (hipEvent timing,
median of N back-to-back launches) on the live buffers of a real step.
    python scripts/kernel_lab.py [--reps 200] [--batch 64]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpi_tensorflow_amd import config as C
from mpi_tensorflow_amd.ops import native, ptr, stream_handle
from mpi_tensorflow_amd.runtime.mnist_engine import NativeMnistEngine
from mpi_tensorflow_amd.utils.data import synthetic_rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--step-only", action="store_true",
                    help="only the graph-replayed step per FC SGD placement (any dtype)")
    ap.add_argument("--rounds", default="0,2", help="FC SGD placements to time (fc_sgd_rounds)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    x, y = synthetic_rows("train", 0, 4096)
    cfg = C.TrainConfig(batch_size=a.batch, graph=False, dtype=a.dtype).validate()
    if a.step_only:
        e = NativeMnistEngine(cfg, x, y, dev)
        step_placements(e, [int(r) for r in a.rounds.split(",")])
        return
    e = NativeMnistEngine(cfg, x, y, dev, fc1_feature_major=True)  # + the a2ft lab buffer
    e.train(5)
    e.forward_backward_only()
    torch.cuda.synchronize()
    Cn = native()
    k = Cn.mnist
    b, B, lay = e.bufs, e.B, e.layout
    W = lambda n: ptr(e.params) + 4 * lay.offsets[n]
    G = lambda n: ptr(e.grads) + 4 * lay.offsets[n]
    s = stream_handle()
    ops = {
        "conv1_fwd": lambda: k.conv1_fwd(ptr(e.train_x), ptr(e.step_dev), e.n_local, B, W("conv1_weight"),
                                         W("conv1_bias"), ptr(b["a1"]), ptr(b["idx1"]), s, ptr(b["a1pf"])),
        "conv2_fwd": lambda: k.conv2_fwd(ptr(b["a1"]), B, W("conv2_weight"), W("conv2_bias"), ptr(b["a2"]),
                                         ptr(b["idx2"]), ptr(b["w2t"]), s),
        "conv2_wino_w": lambda: k.conv2_wino_weights(W("conv2_weight"), ptr(b["wino_u"]), 0, s),
        "conv2_fwd_wino": lambda: k.conv2_fwd_wino(ptr(b["a1"]), B, W("conv2_weight"), ptr(b["wino_u"]),
                                                   W("conv2_bias"), ptr(b["a2"]), ptr(b["idx2"]),
                                                   ptr(b["w2t"]), s),
        "conv12_fwd_wino": lambda: k.conv12_fwd_wino(
            ptr(e.train_x), ptr(e.step_dev), e.n_local, B, W("conv1_weight"), W("conv1_bias"),
            ptr(b["a1"]), ptr(b["a1pf"]), ptr(b["idx1"]), W("conv2_weight"), ptr(b["wino_u"]),
            W("conv2_bias"), ptr(b["a2"]), ptr(b["idx2"]), 0, s, 0, ptr(b["a2ft"])),
        "conv2_bwd_data_wino": lambda: k.conv2_bwd_data_wino(ptr(b["dy2"]), ptr(b["wino_ud"]), ptr(b["a1"]),
                                                             B, ptr(b["da1m"]), s),
        "fc1_fwd": lambda: k.fc1_fwd_train(ptr(b["a2"]), W("fc1_weight"), B, ptr(b["fc1_part"]), s),
        "fc1_fwd_t": lambda: k.fc1_fwd_train_t(ptr(b["a2ft"]), W("fc1_weight"), B, ptr(b["fc1_part"]),
                                               s),
        "fc_head": lambda: k.fc_head_train(ptr(b["fc1_part"]), W("fc1_bias"), W("fc2_weight"), W("fc2_bias"),
                                           ptr(e.train_y), e.n_local, ptr(e.step_dev), B, 0.5, 1, 0, 0.01, 0.95,
                                           ptr(b["hd"]), ptr(b["dh"]), ptr(b["dlog"]), ptr(b["loss_rows"]),
                                           ptr(e.lr_dev), 0, s),
        "fc_head[8]": lambda: k.fc_head_train(ptr(b["fc1_part"]), W("fc1_bias"), W("fc2_weight"),
                                              W("fc2_bias"), ptr(e.train_y), e.n_local, ptr(e.step_dev),
                                              B, 0.5, 1, 0, 0.01, 0.95, ptr(b["hd"]), ptr(b["dh"]),
                                              ptr(b["dlog"]), ptr(b["loss_rows"]), ptr(e.lr_dev), 0, s,
                                              k.fc1_train_t_splits()),
        "fc1_bwd": lambda: k.fc1_bwd(ptr(b["a2"]), ptr(b["idx2"]), ptr(b["dh"]), ptr(b["hd"]), ptr(b["dlog"]),
                                     W("fc1_weight"), B, G("fc1_weight"), G("fc1_bias"), G("fc2_weight"),
                                     G("fc2_bias"), ptr(b["dy2"]), ptr(b["dy2t"]), s),
        "fc1_bwd[dX]": lambda: k.fc1_bwd(ptr(b["a2"]), ptr(b["idx2"]), ptr(b["dh"]), ptr(b["hd"]),
                                         ptr(b["dlog"]), W("fc1_weight"), B, G("fc1_weight"),
                                         G("fc1_bias"), G("fc2_weight"), G("fc2_bias"), ptr(b["dy2"]),
                                         ptr(b["dy2t"]), s, 1),
        "fc1_bwd[dW]": lambda: k.fc1_bwd(ptr(b["a2"]), ptr(b["idx2"]), ptr(b["dh"]), ptr(b["hd"]),
                                         ptr(b["dlog"]), W("fc1_weight"), B, G("fc1_weight"),
                                         G("fc1_bias"), G("fc2_weight"), G("fc2_bias"), ptr(b["dy2"]),
                                         ptr(b["dy2t"]), s, 2),
        "fc1_bwd[small]": lambda: k.fc1_bwd(ptr(b["a2"]), ptr(b["idx2"]), ptr(b["dh"]), ptr(b["hd"]),
                                            ptr(b["dlog"]), W("fc1_weight"), B, G("fc1_weight"),
                                            G("fc1_bias"), G("fc2_weight"), G("fc2_bias"),
                                            ptr(b["dy2"]), ptr(b["dy2t"]), s, 4),
        "fc1_bwd[dX,no-t]": lambda: k.fc1_bwd(ptr(b["a2"]), ptr(b["idx2"]), ptr(b["dh"]), ptr(b["hd"]),
                                              ptr(b["dlog"]), W("fc1_weight"), B, G("fc1_weight"),
                                              G("fc1_bias"), G("fc2_weight"), G("fc2_bias"),
                                              ptr(b["dy2"]), 0, s, 1),
        "conv2_bwd_data": lambda: k.conv2_bwd_data_l2(ptr(b["dy2t"]), ptr(b["w2t"]), ptr(b["a1"]), B,
                                                      ptr(b["da1m"]), s),
        "conv2_bwd_filter": lambda: k.conv2_bwd_filter(ptr(b["a1pf"]), ptr(b["dy2"]), B, ptr(b["part2"]), s),
        "conv2_bwd_filter_wino": lambda: k.conv2_bwd_filter_wino(ptr(b["a1pf"]), ptr(b["dy2"]), B,
                                                                  ptr(b["part2"]), s),
        "grad_finalize_wino": lambda: k.grad_finalize(ptr(b["part2"]), k.conv2_wino_filter_groups(B),
                                                      ptr(b["part1"]), k.conv1_filter_blocks(B, 1),
                                                      G("conv2_weight"), G("conv2_bias"),
                                                      G("conv1_weight"), G("conv1_bias"), s),
        "conv1_bwd_filter": lambda: k.conv1_bwd_filter(ptr(e.train_x), ptr(e.step_dev), e.n_local, B,
                                                       ptr(b["da1m"]), ptr(b["idx1"]), ptr(b["part1"]), s),
        "grad_finalize": lambda: k.grad_finalize(ptr(b["part2"]), k.conv2_filter_splits(B), ptr(b["part1"]),
                                                 k.conv1_filter_blocks(B), G("conv2_weight"), G("conv2_bias"),
                                                 G("conv1_weight"), G("conv1_bias"), s),
        "sgd": lambda: Cn.optim.sgd_momentum(ptr(e.params), ptr(e.grads), ptr(e.mom), lay.total,
                                             lay.l2_range()[1], 5e-4, 0.9, 1.0, ptr(e.lr_dev), 0.0, 0, s),
    }
    total = 0.0
    print(f"{'kernel':20s} {'median_us':>10s} {'min_us':>8s}")
    for name, fn in ops.items():
        ts = []
        for _ in range(10):
            fn()
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1000.0)
        ts.sort()
        med = ts[len(ts) // 2]
        total += med
        print(f"{name:20s} {med:10.2f} {ts[0]:8.2f}")
    print(f"{'sum':20s} {total:10.2f}")
    # whole step, eager (two streams live)
    e.use_graph = False
    e.train(20)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    e.train(300)
    e1.record()
    e1.synchronize()
    print(f"step (eager): {e0.elapsed_time(e1) * 1000.0 / 300:.2f} us")
    # whole step, graph replay
    e.cfg.graph = True
    e.use_graph = True
    e.capture(50)
    e.train(50)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    e.train(500)
    e1.record()
    e1.synchronize()
    print(f"step (graph replay): {e0.elapsed_time(e1) * 1000.0 / 500:.2f} us")
    step_placements(e, [int(r) for r in a.rounds.split(",")])


def step_placements(e, rounds_list=(0, 2)):
    """Graph-replayed step with the single-rank FC momentum SGD in the conv2
    bwd-data launch (rounds > 0) or in the final SGD launch (rounds = 0)."""
    e.cfg.graph = True
    e.use_graph = True
    for rounds in rounds_list:
        e.exe.set_fc_sgd_rounds(rounds)
        e._graphs.clear()
        e.capture(50)
        e.train(50)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        e.train(500)
        e1.record()
        e1.synchronize()
        print(f"step (graph replay, fc_sgd_rounds={rounds}): "
              f"{e0.elapsed_time(e1) * 1000.0 / 500:.2f} us")


if __name__ == "__main__":
    main()
