"""A/B of the ResNet-18 s2d stem forward loaders (lab): S2dLoaderPre (every
K tile requested at once) vs S2dLoader (one tile ahead), B = 32, 224 x 224,
with the BatchNorm statistics epilogue; hipEvent time per launch over 200
back-to-back launches, alternating 3 rounds.  Run under rocprofv3 for the
kernel times.
    python scripts/s2d_lab.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpi_tensorflow_amd.ops import functional as Fn  # noqa: E402
from mpi_tensorflow_amd.ops import native, ptr, stream_handle  # noqa: E402

ops = native().ops
dev = torch.device("cuda")
N, H, K = 32, 224, 64
x = torch.randn(N, H, H, 3, device=dev)
w = torch.randn(7, 7, 3, K, device=dev) * 0.1
sh = ops.ConvShape(N, H, H, 3, K, 7, 7, 2, 3)
si = Fn._s2d_shape(sh)
s = stream_handle()
xs = torch.empty(N * si.H * si.W * 16, dtype=torch.bfloat16, device=dev)
ops.s2d_stem_input(ptr(x), N, H, H, sh.OH, sh.OW, ptr(xs), s)
wt8 = torch.empty(K * 256, dtype=torch.bfloat16, device=dev)
ops.s2d_stem_weight(ptr(w), K, ptr(wt8), s)
s1 = ops.ConvShape(N, sh.OH, sh.OW, 256, K, 1, 1, 1, 0)
rows = ops.conv_fwd_stem_stats_rows(s1)
shift = torch.zeros(K, device=dev)
y = torch.empty(N, sh.OH, sh.OW, K, dtype=torch.bfloat16, device=dev)
part = torch.empty(2 * K * rows, device=dev)
REPS = 200
for rnd in range(3):
    for pre in (False, True):
        ops.s2d_stem_set_preload(pre)
        for _ in range(10):
            ops.conv_fwd_s2d_stem_bf16(si, ptr(xs), ptr(wt8), ptr(y), s, ptr(part), rows, ptr(shift))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(REPS):
            ops.conv_fwd_s2d_stem_bf16(si, ptr(xs), ptr(wt8), ptr(y), s, ptr(part), rows, ptr(shift))
        e1.record()
        torch.cuda.synchronize()
        print(f"round {rnd} preload={pre}: {1000 * e0.elapsed_time(e1) / REPS:.2f} us/launch",
              flush=True)
ops.s2d_stem_set_preload(True)
