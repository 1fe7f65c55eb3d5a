"""Per-(kernel, grid) breakdown of a rocprofv3 kernel trace, in us per step.
    python scripts/prof_grid.py gpurun_out/prof/x_results.db STEPS [TOP]"""
import sqlite3
import sys
from collections import defaultdict

con = sqlite3.connect(sys.argv[1])
steps = int(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
agg = defaultdict(lambda: [0, 0.0])
for n, gx, gy, gz, d in con.execute("select name,grid_x,grid_y,grid_z,duration from kernels"):
    a = agg[(n[:64], gx, gy, gz)]
    a[0] += 1
    a[1] += d / 1000.0
tot = sum(v[1] for v in agg.values())
print(f"{'kernel':64s} {'grid':>18s} {'calls':>6s} {'us/step':>9s} {'mean_us':>8s}")
for (n, gx, gy, gz), (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{n:64s} {f'{gx}x{gy}x{gz}':>18s} {c:6d} {t / steps:9.1f} {t / c:8.1f}")
print(f"total kernel time {tot / steps:.1f} us/step over {steps} steps")
