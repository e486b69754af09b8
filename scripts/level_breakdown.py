"""Per-level kernel time of the last tree in a rocprofv3 kernel trace (deep-tree engines)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
keys = ["split_find", "seg_direct", "hist_build_seg", "hist_build_kernel", "hist_reduce", "level_finalize", "level_close",
        "part_scatter", "zero_slots", "part_count", "node_best", "lf_", "seg_colmajor"]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
seq = [(r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, r["Grid_Size_X"]) for r in rows]
LEVEL = ("split_find", "seg_direct")   # one of these per level (direct mode replaces split_find)
idx = [i for i, (n, d, g) in enumerate(seq) if any(k in n for k in LEVEL)]
depth = int(sys.argv[2]) if len(sys.argv) > 2 else 20
start = idx[-depth]
lvl, out = -1, {}
for n, d, g in seq[start - 3:]:
    for k in keys:
        if k in n:
            if k in LEVEL:
                lvl += 1
            e = out.setdefault(lvl, {})
            e[k] = e.get(k, 0.0) + d
            if k in LEVEL:
                e["grid"] = g
tot = 0.0
for lv in sorted(out):
    s = sum(v for k, v in out[lv].items() if k != "grid")
    tot += s
    print(lv, round(s, 1), {k: (round(v, 1) if k != "grid" else v) for k, v in out[lv].items()})
print("total us", round(tot, 1))
