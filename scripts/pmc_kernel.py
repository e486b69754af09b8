#!/usr/bin/env python3
"""Per-dispatch counters of one kernel from rocprofv3 --pmc CSVs: pmc_kernel.py DIR NAME_SUBSTR"""
import csv
import glob
import sys
from collections import OrderedDict, defaultdict

root, name = sys.argv[1], sys.argv[2]
rows = defaultdict(OrderedDict)
for f in glob.glob(root + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if name not in (r.get("Kernel_Name") or ""):
            continue
        did = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)
        rows[did][r["Counter_Name"]] = float(r["Counter_Value"])
ids = sorted(rows)
names = sorted({c for d in rows.values() for c in d})
print("dispatch".ljust(10), " ".join(n[:20].rjust(20) for n in names))
for i in ids[-12:]:
    print(str(i).ljust(10), " ".join(f"{rows[i].get(n, float('nan')):.4g}".rjust(20) for n in names))
