"""Times the 3x3 stride-1 bf16 filter gradient (conv_bf16.hip wgrad3) on the
ResNet-18 layer shapes at batch B, in a 20-launch hipGraph; checks it against
torch on the first rep.
    python scripts/wgrad3_lab.py [B]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from mpi_tensorflow_amd.ops import native, ptr, stream_handle

B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
g = native().ops
dev = torch.device("cuda:0")
tot = 0.0
for H, C, cnt in ((56, 64, 4), (28, 128, 3), (14, 256, 3), (7, 512, 3)):
    sh = g.ConvShape(B, H, H, C, C, 3, 3, 1, 1)
    x = torch.randn(B, H, H, C, device=dev)
    dy = torch.randn(B, H, H, C, device=dev)
    xb, dyb = x.to(torch.bfloat16), dy.to(torch.bfloat16)
    dw = torch.empty(3, 3, C, C, device=dev)
    ws = torch.empty(max(g.conv_ws_floats(sh, False), 4), device=dev)
    s = stream_handle()
    g.conv_bwd_filter(sh, ptr(x), ptr(dy), ptr(ws), ptr(dw), s, True, ptr(xb), ptr(dyb))
    torch.cuda.synchronize()
    ref = torch.nn.grad.conv2d_weight(xb.float().permute(0, 3, 1, 2), (C, C, 3, 3),
                                      dyb.float().permute(0, 3, 1, 2), padding=1)
    err = ((dw.permute(3, 2, 0, 1) - ref).abs().max() / ref.abs().max()).item()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(20):
            g.conv_bwd_filter(sh, ptr(x), ptr(dy), ptr(ws), ptr(dw), stream_handle(), True, ptr(xb),
                              ptr(dyb))
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        gr.replay()
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) * 1000 / 100
    tot += us * cnt
    print(f"H{H:3d} C{C:3d}: {us:7.2f} us/call  x{cnt}  rel.err {err:.1e}", flush=True)
print(f"total per step (13 convs): {tot:.1f} us")
