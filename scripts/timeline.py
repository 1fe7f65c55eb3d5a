"""Print a window of a rocprofv3 kernel trace as a timeline (start, duration,
gap to the previous kernel on the same queue, queue, name).
    python scripts/timeline.py gpurun_out/x/x_results.db [--from-end N] [--count M]"""
import argparse
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--from-end", type=int, default=200)
ap.add_argument("--count", type=int, default=40)
a = ap.parse_args()
con = sqlite3.connect(a.db)
rows = list(con.execute("select name, start, end, queue_id from kernels order by start"))
rs = rows[-a.from_end:][: a.count]
t0 = rs[0][1]
last_end = {}
for n, s, e, q in rs:
    gap = (s - last_end[q]) / 1000 if q in last_end else 0.0
    last_end[q] = e
    print(f"{(s - t0) / 1000:9.2f} {(e - s) / 1000:8.2f} gap {gap:7.2f} q{q} {n.split('(')[0][-60:]}")
