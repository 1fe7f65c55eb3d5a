"""Cost of the BatchNorm-statistics epilogue on the bf16 ResNet-18 convs:
times conv2d(out_bf16=True) with and without a BnLink (epilogue statistics), back to back.
    python scripts/conv_stats_lab.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpi_tensorflow_amd.ops import functional as Fn


def _param(t):
    p = Fn.Param.__new__(Fn.Param)
    p.value, p.grad_view, p.wtb, p.wtb_d = t, torch.zeros_like(t), None, None
    return p


def main():
    dev = torch.device("cuda")
    Fn.set_conv_bf16(True)
    for (N, H, C, K, R, st, pad) in [(32, 56, 64, 64, 3, 1, 1), (32, 28, 128, 128, 3, 1, 1),
                                     (32, 14, 256, 256, 3, 1, 1), (32, 7, 512, 512, 3, 1, 1),
                                     (32, 56, 64, 128, 3, 2, 1)]:
        x = torch.randn(N, H, H, C, device=dev)
        w = _param(torch.randn(R, R, C, K, device=dev) * 0.05)
        rm = torch.zeros(K, device=dev)
        res = []
        for shift in (None, rm):
            with torch.no_grad():
                for _ in range(5):
                    Fn.conv2d(x, w, None, st, pad, out_bf16=True, bn_out=None if shift is None else Fn.BnLink(shift))
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(50):
                    Fn.conv2d(x, w, None, st, pad, out_bf16=True, bn_out=None if shift is None else Fn.BnLink(shift))
                b.record()
                b.synchronize()
                res.append(a.elapsed_time(b) * 1000 / 50)
        print(f"N{N} H{H} C{C} K{K} R{R} s{st}: plain {res[0]:.2f} us, with stats {res[1]:.2f} us",
              flush=True)


if __name__ == "__main__":
    main()
