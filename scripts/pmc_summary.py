#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSV output: mean counter value per kernel (top kernels)."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
files = glob.glob(root + "/**/*counter_collection.csv", recursive=True)
if not files:
    print("no counter_collection.csv under", root)
    sys.exit(0)
acc = defaultdict(lambda: defaultdict(list))
for f in files:
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name") or row.get("KernelName") or "?"
        c = row.get("Counter_Name") or row.get("CounterName")
        v = row.get("Counter_Value") or row.get("CounterValue")
        try:
            acc[k[:60]][c].append(float(v))
        except (TypeError, ValueError):
            pass
names = sorted({c for d in acc.values() for c in d})
print("kernel".ljust(60), " ".join(n[:22].rjust(22) for n in names))
for k, d in sorted(acc.items(), key=lambda kv: -max((sum(v) / len(v) for v in kv[1].values()), default=0))[:25]:
    print(k.ljust(60), " ".join((f"{sum(d[n]) / len(d[n]):.4g}" if d.get(n) else "-").rjust(22) for n in names))
