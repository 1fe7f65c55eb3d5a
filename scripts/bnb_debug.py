"""Debug lab: the BatchNorm backward sums a dgrad epilogue / slab reduction
writes (BnBwdStats) vs the same sums in torch, per channel.
    python scripts/bnb_debug.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpi_tensorflow_amd.ops import native, ptr, stream_handle


def run(N, H, Cin, K, stride, relu):
    C = native()
    g = C.ops
    dev = torch.device("cuda:0")
    gen = torch.Generator().manual_seed(3)
    OH = (H + 2 - 3) // stride + 1
    sh = g.ConvShape(N, H, H, Cin, K, 3, 3, stride, 1)
    w = (torch.randn(3, 3, Cin, K, generator=gen) * 0.05).to(dev)
    dyb = torch.randn(N, OH, OH, K, generator=gen).to(torch.bfloat16).to(dev)
    x = (torch.randn(N, H, H, Cin, generator=gen) * 2 + 0.5).to(torch.bfloat16).to(dev)
    y = torch.randn(N, H, H, Cin, generator=gen).to(torch.bfloat16).to(dev)
    mean = torch.randn(Cin, generator=gen).to(dev)
    rstd = (torch.rand(Cin, generator=gen) + 0.5).to(dev)
    ws = torch.zeros(max(g.conv_ws_floats(sh, False), 4), device=dev)
    dx = torch.zeros(N, H, H, Cin, device=dev)
    P = g.conv_bwd_data_stats_rows(sh)
    part = torch.full((2 * Cin * P,), float("nan"), device=dev)
    s = stream_handle()
    g.conv_bwd_data(sh, 0, ptr(w), ptr(dx), ptr(ws), s, True, ptr(dyb), 0, 0, ptr(part), P,
                    ptr(x), ptr(y), ptr(mean), ptr(rstd), relu)
    torch.cuda.synchronize()
    t = part.view(2, Cin // 64, P, 64).sum(2).reshape(2, Cin)
    d = dx * ((y.float() > 0) if relu else 1.0)
    ref1 = d.sum((0, 1, 2))
    ref2 = (d * (x.float() - mean) * rstd).sum((0, 1, 2))
    e1 = ((t[0] - ref1).abs() / ref1.abs().clamp_min(1e-3))
    e2 = ((t[1] - ref2).abs() / ref2.abs().clamp_min(1e-3))
    print(f"N={N} H={H} C={Cin} K={K} s={stride} relu={relu} P={P} nan={part.isnan().sum().item()}"
          f" max rel err s1 {e1.max().item():.2e} s2 {e2.max().item():.2e}")
    bad = (e1 > 1e-3).nonzero().flatten().tolist()
    if bad:
        print("  bad channels:", bad[:32])
        print("  got", t[0][bad[:8]].tolist(), "want", ref1[bad[:8]].tolist())


if __name__ == "__main__":
    for args in [(4, 14, 64, 64, 1, True), (4, 7, 512, 512, 1, True), (32, 56, 64, 128, 2, True),
                 (2, 28, 64, 128, 2, True), (2, 28, 64, 128, 2, False), (4, 14, 256, 256, 2, True)]:
        run(*args)
