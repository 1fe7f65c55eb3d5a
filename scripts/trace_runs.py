"""Splits a rocprofv3 SQLite kernel trace into runs of consecutive dispatches
of one kernel (a lab script that launches variant A 200 times, then variant B
200 times, ... gives one run per variant) and prints each run's median and
minimum duration, so variants of the SAME kernel are timed on the GPU clock
without the host-side event overhead.
    python scripts/trace_runs.py gpurun_out/lab/run_results.db [--min-count 20]"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    min_count = int(sys.argv[sys.argv.index("--min-count") + 1]) if "--min-count" in sys.argv else 20
    con = sqlite3.connect(db)
    cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
    ki = {c: i for i, c in enumerate(cols)}
    name_col = "kernel_name" if "kernel_name" in ki else "name"
    rows = con.execute("select * from kernels order by start").fetchall()
    runs = []
    for r in rows:
        n = r[ki[name_col]]
        d = (r[ki["end"]] - r[ki["start"]]) / 1000.0
        if runs and runs[-1][0] == n:
            runs[-1][1].append(d)
        else:
            runs.append([n, [d]])
    print(f"{'run':>4s} {'kernel':70s} {'count':>6s} {'median_us':>10s} {'min_us':>8s}")
    k = 0
    for n, ds in runs:
        if len(ds) < min_count:
            continue
        ds.sort()
        short = n if len(n) <= 70 else n[:67] + "..."
        print(f"{k:4d} {short:70s} {len(ds):6d} {ds[len(ds) // 2]:10.2f} {ds[0]:8.2f}")
        k += 1


if __name__ == "__main__":
    main()
