"""Times the conv2 kernels of the native MNIST step back to back (N launches
between two events, so launch latency is amortised as in graph replay):
direct vs Winograd forward / bwd-data / filter gradient, and the filter
transform.
    python scripts/wino_lab.py [--reps 200]"""
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
    ap.add_argument("--only", default="")
    ap.add_argument("--phases", action="store_true", help="per-phase s_memtime of the Winograd wgrad")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    x, y = synthetic_rows("train", 0, 4096)
    cfg = C.TrainConfig(graph=False).validate()
    e = NativeMnistEngine(cfg, x, y, dev)
    e.train(3)
    e.forward_backward_only()
    torch.cuda.synchronize()
    k = native().mnist
    b, B, lay = e.bufs, e.B, e.layout
    W = lambda n: ptr(e.params) + 4 * lay.offsets[n]  # noqa: E731
    s = stream_handle()
    k.conv2_wino_weights(W("conv2_weight"), ptr(b["wino_u"]), ptr(b["wino_ud"]), s)
    w2t = torch.empty(25 * 64 * 32, device=dev)
    ops = {
        "conv2_fwd(direct)": lambda: k.conv2_fwd(ptr(b["a1"]), B, W("conv2_weight"), W("conv2_bias"),
                                                 ptr(b["a2"]), ptr(b["idx2"]), ptr(w2t), s),
        "conv2_fwd(wino)": lambda: k.conv2_fwd_wino(ptr(b["a1"]), B, W("conv2_weight"), ptr(b["wino_u"]),
                                                    W("conv2_bias"), ptr(b["a2"]), ptr(b["idx2"]), 0, s),
        "wino_weights": lambda: k.conv2_wino_weights(W("conv2_weight"), ptr(b["wino_u"]),
                                                     ptr(b["wino_ud"]), s),
        "bwd_data(direct)": lambda: k.conv2_bwd_data_l2(ptr(b["dy2t"]), ptr(w2t), ptr(b["a1"]), B,
                                                        ptr(b["da1m"]), s),
        "wgrad(direct)": lambda: k.conv2_bwd_filter(ptr(b["a1pf"]), ptr(b["dy2"]), B, ptr(b["part2"]), s),
        "wgrad(wino)": lambda: k.conv2_bwd_filter_wino(ptr(b["a1pf"]), ptr(b["dy2"]), B, ptr(b["part2"]), s),
        "bwd_data(wino)": lambda: k.conv2_bwd_data_wino(ptr(b["dy2"]), ptr(b["wino_ud"]), ptr(b["a1"]),
                                                        B, ptr(b["da1m"]), s),
    }
    if a.phases:
        G = k.conv2_wino_filter_groups(B)
        nw = 12
        prof = torch.zeros(8 * G * nw * 5, dtype=torch.int64, device=dev)
        for _ in range(5):
            k.conv2_bwd_filter_wino_prof(ptr(b["a1pf"]), ptr(b["dy2"]), B, ptr(b["part2"]), ptr(prof), s)
        torch.cuda.synchronize()
        t = prof.view(8 * G, nw, 5).double()
        t0 = t[..., 0].min()
        d = t[..., 1:] - t[..., :-1]
        names = ["staging", "main loop", "db + S_a", "dW + stores"]
        print("wgrad(wino) phases, cycles per wave: mean / max")
        for i, nm in enumerate(names):
            print(f"  {nm:12s} {d[..., i].mean().item():9.0f} {d[..., i].max().item():9.0f}")
        print(f"  span (first start -> last end) {(t[..., 4].max() - t0).item():.0f} cycles; "
              f"block start spread {(t[..., 0].max() - t0).item():.0f}")
    if a.phases:
        nb, nw = B * 4, 8
        W_ = lambda n: ptr(e.params) + 4 * lay.offsets[n]  # noqa: E731
        pf = torch.zeros(nb * nw * 5, dtype=torch.int64, device=dev)
        pb = torch.zeros(nb * nw * 7, dtype=torch.int64, device=dev)
        part1 = torch.zeros(B * 4 * 832, device=dev)
        for _ in range(5):
            k.conv12_fwd_wino(ptr(e.train_x), ptr(e.step_dev), e.n_local, B, W_("conv1_weight"),
                              W_("conv1_bias"), ptr(b["a1"]), ptr(b["a1pf"]), ptr(b["idx1"]),
                              W_("conv2_weight"), ptr(b["wino_u"]), W_("conv2_bias"), ptr(b["a2"]),
                              ptr(b["idx2"]), 0, s, ptr(pf))
            k.conv2_bwd_data_wino_prof(ptr(b["dy2"]), ptr(b["wino_ud"]), ptr(b["a1"]), B,
                                       ptr(b["da1m"]), ptr(e.train_x), ptr(e.step_dev), e.n_local,
                                       ptr(b["idx1"]), ptr(part1), ptr(pb), s)
        torch.cuda.synchronize()
        for nm, t, names in (("conv12_fwd(wino)", pf.view(nb, nw, 5).double(),
                              ["conv1 -> halo", "input transform", "products", "sums + epilogue"]),
                             ("bwd_data(wino)+c1", pb.view(nb, nw, 7).double(),
                              ["h0 transform", "h0 products", "h1 transform", "h1 products",
                               "sums + dA1", "conv1 wgrad"])):
            t0 = t[..., 0].min()
            d = t[..., 1:] - t[..., :-1]
            print(f"{nm} phases, cycles per wave: mean / max")
            for i, ph in enumerate(names):
                print(f"  {ph:16s} {d[..., i].mean().item():9.0f} {d[..., i].max().item():9.0f}")
            print(f"  span (first start -> last end) {(t[..., -1].max() - t0).item():.0f} cycles; "
                  f"block start spread {(t[..., 0].max() - t0).item():.0f}")
    for name, fn in ops.items():
        if a.only and a.only not in name:
            continue
        for _ in range(10):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        e1.synchronize()
        print(f"{name:22s} {e0.elapsed_time(e1) * 1000.0 / a.reps:8.2f} us/launch (back to back)",
              flush=True)


if __name__ == "__main__":
    main()
