"""Summarise a rocprofv3 SQLite kernel trace: per-kernel count, total, mean,
and the average gap between consecutive dispatches (launch/boundary cost).
    python scripts/prof_summary.py gpurun_out/prof/run_results.db [--last N]"""
import sqlite3
import sys
from collections import defaultdict

db = sys.argv[1]
con = sqlite3.connect(db)
cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
rows = con.execute("select * from kernels order by start").fetchall()
ki = {c: i for i, c in enumerate(cols)}
name_col = "kernel_name" if "kernel_name" in ki else ("name" if "name" in ki else None)
agg = defaultdict(lambda: [0, 0.0])
for r in rows:
    n = r[ki[name_col]]
    d = (r[ki["end"]] - r[ki["start"]]) / 1000.0
    a = agg[n]
    a[0] += 1
    a[1] += d
tot = sum(v[1] for v in agg.values())
print(f"{'kernel':90s} {'calls':>7s} {'total_us':>11s} {'mean_us':>9s} {'%':>6s}")
for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    short = n if len(n) <= 90 else n[:87] + "..."
    print(f"{short:90s} {c:7d} {t:11.1f} {t / c:9.2f} {100 * t / tot:6.1f}")
print(f"total kernel time {tot:.1f} us over {len(rows)} dispatches")
if len(rows) > 2:
    span = (rows[-1][ki["end"]] - rows[0][ki["start"]]) / 1000.0
    print(f"wall span first->last dispatch {span:.1f} us; busy fraction {tot / span:.3f}")
