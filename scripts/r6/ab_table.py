#!/usr/bin/env python3
"""Median / spread table of drf_deep_ab.py JSON lines: ab_table.py DIR ARM [ARM ...]
(files DIR/drf_<ARM>_<rep>.jsonl; the warm second fit of each process is the sample)."""
import glob
import json
import statistics as S
import sys

d = sys.argv[1]
for arm in sys.argv[2:]:
    v = []
    for f in sorted(glob.glob(f"{d}/drf_{arm}_*.jsonl")):
        rows = [json.loads(x) for x in open(f) if x.strip()]
        v += [(r["ms_per_tree"], r["auc"]) for r in rows if r.get("rep") == 1]
    t = [x[0] for x in v]
    print(f"{arm:12s} ms/tree median {S.median(t):6.2f} [{min(t):.2f}, {max(t):.2f}]  runs {', '.join(f'{x:.2f}' for x in t)}"
          f"  auc {sorted({x[1] for x in v})}")
