"""Per-kernel, per-grid averages of rocprofv3 --pmc results (rocpd SQLite,
`counters_collection`), SQ counters also per wave.
    python scripts/pmc_summary.py gpurun_out/pmc1 [gpurun_out/pmc2 ...] [--match conv3]"""
import glob
import sqlite3
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:] if not a.startswith("--")]
match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else ""
for d in args:
    if d == match:
        continue
    db = glob.glob(d + "/*.db")[0]
    con = sqlite3.connect(db)
    rows = con.execute("select kernel_name, grid_size, counter_name, value from counters_collection")
    agg = defaultdict(lambda: defaultdict(list))
    for name, grid, cn, v in rows:
        if match in name:
            agg[(name.split("(")[0][-60:], grid)][cn].append(v)
    print(d)
    for (name, grid), cs in sorted(agg.items()):
        waves = cs.get("SQ_WAVES")
        w = sum(waves) / len(waves) if waves else None
        vals = []
        for cn, vs in sorted(cs.items()):
            m = sum(vs) / len(vs)
            per_wave = f"/wave {m / w:,.0f}" if (w and cn.startswith("SQ_") and cn != "SQ_WAVES") else ""
            vals.append(f"{cn}={m:,.0f}{per_wave}")
        print(f"  {name} grid={grid}: " + "; ".join(vals))
