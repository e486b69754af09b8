#!/usr/bin/env python3
"""Counter totals per kernel family from rocprofv3 --pmc CSV directories:
pmc_by_kernel.py DIR [DIR ...] -> one table (sums over every dispatch of the
family) plus per-wave / ratio columns."""
import csv
import glob
import re
import sys
from collections import defaultdict

# a counter collected in several passes (SQ_WAVES, SQ_WAVE_CYCLES as the
# per-pass anchors) is taken from the first pass that has it
tot = defaultdict(dict)
disp = defaultdict(set)
for root in sys.argv[1:]:
    part = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(root + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name") or ""
            fam = re.sub(r"[<(].*", "", name).replace("void ", "").strip()
            part[fam][r["Counter_Name"]] += float(r["Counter_Value"])
            if root == sys.argv[1]:
                disp[fam].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
    for fam, d in part.items():
        for c, v in d.items():
            tot[fam].setdefault(c, v)
fams = sorted(tot, key=lambda k: -tot[k].get("SQ_WAVE_CYCLES", tot[k].get("SQ_BUSY_CYCLES", 0.0)))
names = sorted({c for d in tot.values() for c in d})
print("family".ljust(34), "disp".rjust(6), " ".join(n[:22].rjust(22) for n in names))
for k in fams[:25]:
    print(k[:34].ljust(34), str(len(disp[k])).rjust(6), " ".join(f"{tot[k].get(n, float('nan')):.4g}".rjust(22) for n in names))
print()
print("family".ljust(34), "valu/wave  vmemrd/wave  lds/wave  salu/wave  wait_any/wave_cyc  lds_conflict/idx_active  tcc_hit")
for k in fams[:25]:
    d = tot[k]
    w = d.get("SQ_WAVES", float("nan")) or float("nan")
    def g(n):
        v = d.get(n, float("nan"))
        return float("nan") if v == 0 else v
    hit = g("TCC_HIT_sum") / (g("TCC_HIT_sum") + g("TCC_MISS_sum")) if "TCC_HIT_sum" in d else float("nan")
    print(k[:34].ljust(34), f"{g('SQ_INSTS_VALU') / w:9.1f} {g('SQ_INSTS_VMEM_RD') / w:11.1f} {g('SQ_INSTS_LDS') / w:9.1f}"
          f" {g('SQ_INSTS_SALU') / w:10.1f} {g('SQ_WAIT_INST_ANY') / g('SQ_WAVE_CYCLES'):18.3f}"
          f" {g('SQ_LDS_BANK_CONFLICT') / g('SQ_LDS_IDX_ACTIVE'):24.3f} {hit:8.3f}")
