#!/usr/bin/env python3
"""Per-dispatch rocprofv3 --pmc table for the last N dispatches (one GBM step).

    python3 scripts/pmc_dispatch.py OUTDIR [N] [kernel-substring ...]

Prints, in dispatch order, every counter of the run per dispatch plus the
derived GB/s when FETCH_SIZE / WRITE_SIZE (KB) and the kernel trace are present.
"""
import csv
import glob
import sys
from collections import OrderedDict


def main():
    root = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    keep = sys.argv[3:]
    files = glob.glob(root + "/**/*counter_collection.csv", recursive=True)
    if not files:
        print("no counter_collection.csv under", root)
        return
    rows = OrderedDict()
    names = []
    for f in files:
        for r in csv.DictReader(open(f)):
            did = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)
            k = r.get("Kernel_Name") or "?"
            c = r.get("Counter_Name")
            if c not in names:
                names.append(c)
            d = rows.setdefault(did, {"kernel": k, "grid": r.get("Grid_Size", ""), "wg": r.get("Workgroup_Size", "")})
            d[c] = d.get(c, 0.0) + float(r.get("Counter_Value") or 0)
    ids = sorted(rows)[-n:]
    print(f"{'kernel':52s} {'grid':>9s} {'wg':>5s} " + " ".join(f"{c[:20]:>20s}" for c in names))
    for i in ids:
        d = rows[i]
        k = d["kernel"].replace("void ", "")[:52]
        if keep and not any(s in k for s in keep):
            continue
        print(f"{k:52s} {d['grid']:>9s} {d['wg']:>5s} " + " ".join(f"{d.get(c, 0):20.4g}" for c in names))


if __name__ == "__main__":
    main()
