"""Per-kernel averages of rocprofv3 --pmc CSV output (one dispatch = one row
per counter).  python scripts/pmc_summary.py <dir-with-*_counter_collection.csv>"""
import csv
import glob
import sys
from collections import defaultdict

for d in sys.argv[1:]:
    f = glob.glob(d + "/*counter_collection.csv")[0]
    agg = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-38:]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    names = sorted({c for v in agg.values() for c in v})
    print(d)
    print(f"{'kernel':38s} " + " ".join(f"{n[-14:]:>14s}" for n in names))
    for k, v in agg.items():
        n = len(disp[k])
        if n < 5:
            continue
        print(f"{k:38s} " + " ".join(f"{v[c] / n:14.0f}" for c in names))
