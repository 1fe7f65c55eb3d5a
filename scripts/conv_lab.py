"""Times the generic conv ops (forward / backward-data / backward-filter) on
every distinct ResNet-18 layer shape at batch B, per op and per layer.
    python scripts/conv_lab.py [--batch 32] [--dtype bf16] [--reps 20]
        [--plan vcap=128,ksplit_target=2048,...]
--plan sets fields of the tiled family's TiledPlan (csrc/kernels/ops_generic.h)
for this run only; production always runs the defaults."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from mpi_tensorflow_amd.ops import native, ptr, stream_handle


def shapes(B):
    # (H, Cin, K, R, stride, pad, count per step)
    return [
        (112, 3, 64, 7, 2, 3, 1),
        (56, 64, 64, 3, 1, 1, 4),
        (56, 64, 128, 3, 2, 1, 1), (28, 128, 128, 3, 1, 1, 3), (56, 64, 128, 1, 2, 0, 1),
        (28, 128, 256, 3, 2, 1, 1), (14, 256, 256, 3, 1, 1, 3), (28, 128, 256, 1, 2, 0, 1),
        (14, 256, 512, 3, 2, 1, 1), (7, 512, 512, 3, 1, 1, 3), (14, 256, 512, 1, 2, 0, 1),
    ]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--layers", default=None, help="comma list of shape-table rows to run")
    ap.add_argument("--ops", default="fwd,dgrad,wgrad")
    ap.add_argument("--plan", default="", help="TiledPlan overrides, k=v comma list")
    a = ap.parse_args()
    C = native()
    g = C.ops
    if a.plan:
        plan = g.get_tiled_plan()
        for kv in a.plan.split(","):
            k, v = kv.split("=")
            cur = getattr(plan, k)
            setattr(plan, k, (v not in ("0", "false")) if isinstance(cur, bool) else int(v))
        g.set_tiled_plan(plan)
    bf16 = a.dtype == "bf16"
    dev = torch.device("cuda:0")
    s = stream_handle()
    tot = [0.0, 0.0, 0.0]
    rows = None if a.layers is None else {int(v) for v in a.layers.split(",")}
    want = set(a.ops.split(","))
    for li, (H, Cin, K, R, st, pd, cnt) in enumerate(shapes(a.batch)):
        if rows is not None and li not in rows:
            continue
        Hin = 224 if Cin == 3 else H  # the table's H is the input size (stem: output)
        sh = g.ConvShape(a.batch, Hin, Hin, Cin, K, R, R, st, pd)
        x = torch.randn(a.batch, Hin, Hin, Cin, device=dev)
        w = torch.randn(R, R, Cin, K, device=dev) * 0.05
        y = torch.empty(a.batch, sh.OH, sh.OW, K, device=dev)
        dy = torch.randn_like(y)
        dx = torch.empty_like(x)
        dw = torch.empty_like(w)
        ws = torch.empty(max(g.conv_ws_floats(sh, False), 4) * 2, device=dev)
        # the engine's bf16 twins of x / dY (written by the BN kernels)
        xb = dyb = None
        if bf16 and g.conv_bf16_ok(sh):
            xb, dyb = x.to(torch.bfloat16), dy.to(torch.bfloat16)
        # fp32: the engine's stride-1 dgrad weight copy (ConvWeightCopies
        # f32flip), which the fp32 dgrad and the halo forward read
        wfl = None
        if not bf16 and R > 1 and Cin % 32 == 0 and K % 32 == 0:
            from mpi_tensorflow_amd.ops import functional as Fn
            prm = Fn.Param(w, dw)
            wc = Fn.ConvWeightCopies({"w": prm}, dev, kind="f32flip")
            wc.refresh()
            wfl = prm.wtb_d
        ops = {
            "fwd": lambda: g.conv_fwd(sh, ptr(x), ptr(w), 0, ptr(y), False, ptr(ws), s, bf16,
                                      ptr(xb), ptr(wfl)),
            "dgrad": lambda: g.conv_bwd_data(sh, ptr(dy), ptr(w), ptr(dx), ptr(ws), s, bf16,
                                             ptr(dyb), 0, ptr(wfl)),
            "wgrad": lambda: g.conv_bwd_filter(sh, ptr(x), ptr(dy), ptr(ws), ptr(dw), s, bf16,
                                               ptr(xb), ptr(dyb)),
        }
        line = f"H{Hin:3d} {Cin:3d}->{K:3d} {R}x{R} s{st} x{cnt}:"
        res = []
        for i, (name, fn) in enumerate(ops.items()):
            if (name == "dgrad" and Cin == 3) or name not in want:
                res.append(0.0)
                continue
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(a.reps):
                fn()
            e1.record()
            e1.synchronize()
            us = e0.elapsed_time(e1) * 1000.0 / a.reps
            res.append(us)
            tot[i] += us * cnt
        line += "  " + " ".join(f"{t:7.1f}" for t in res)
        print(line, flush=True)
    t = tot
    print(f"per-step fwd {t[0]:.0f} dgrad {t[1]:.0f} wgrad {t[2]:.0f} total {sum(t):.0f} us")


if __name__ == "__main__":
    main()
