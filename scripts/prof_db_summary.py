#!/usr/bin/env python3
"""Summarise a rocprofv3 SQLite output (rocpd tables): top kernels and the
dispatch timeline between the last two launches of a marker kernel.

    python scripts/prof_db_summary.py <results.db> [marker] [n_lines]
"""
import sqlite3
import sys
from collections import defaultdict

db, marker = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "boost_update")
con = sqlite3.connect(db)
tabs = [r[0] for r in con.execute("select name from sqlite_master where type='table'")]
kd = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
ks = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol"))
names = {r[0]: r[1] for r in con.execute(f"select id, kernel_name from {ks}")}
cols = [r[1] for r in con.execute(f"pragma table_info({kd})")]
rows = con.execute(f"select kernel_id, start, end, grid_size_x, workgroup_size_x from {kd} order by start").fetchall()
tot = defaultdict(lambda: [0, 0])
for k, s, e, g, w in rows:
    tot[names[k]][0] += 1
    tot[names[k]][1] += e - s
allt = sum(v[1] for v in tot.values())
print("== top kernels ==")
for n, (c, d) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:16]:
    print(f"{n[:64]:64s} calls={c:>6d} avg={d / c / 1e3:8.1f}us tot={d / 1e6:8.2f}ms {100 * d / allt:5.1f}%")
idx = [i for i, r in enumerate(rows) if marker in names[r[0]]]
if len(idx) >= 3:
    a, b = idx[-2], idx[-1]
    t0 = rows[a][1]
    print(f"== one step: {(rows[b][1] - t0) / 1e3:.1f} us ==")
    busy = 0
    for k, s, e, g, w in rows[a:b]:
        busy += e - s
        print(f"  +{(s - t0) / 1e3:8.1f}us {(e - s) / 1e3:8.1f}us  {names[k].split('(')[0][:48]}  grid={g} wg={w}")
    print(f"  kernel-busy {busy / 1e3:.1f} us")
