#!/usr/bin/env python3
"""Per-level PMC table of one GBM tree from two rocprofv3 --pmc passes.

    python3 scripts/pmc_levels_table.py PASS1_DIR PASS2_DIR [PASS3_DIR ...]

Every pass ran the same eager (H2OMX_TREE_GRAPH=0) bench, so dispatch k of one
pass is dispatch k of the others.  The table covers the last complete tree
(boost_update .. leaf_finalize): per dispatch FETCH_SIZE / WRITE_SIZE (MB), the
LDS bank-conflict share (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE), LDS wait
per LDS instruction, and each histogram level's fetch relative to level 0.
"""
import csv
import glob
import sys


def load(root):
    files = glob.glob(root + "/**/*counter_collection.csv", recursive=True)
    rows = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            did = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)
            d = rows.setdefault(did, {"kernel": (r.get("Kernel_Name") or "?").replace("void ", ""),
                                      "grid": r.get("Grid_Size", "")})
            c = r.get("Counter_Name")
            d[c] = d.get(c, 0.0) + float(r.get("Counter_Value") or 0)
    return [rows[k] for k in sorted(rows)]


def last_tree(disp):
    ends = [i for i, d in enumerate(disp) if d["kernel"].startswith("leaf_finalize")]
    if not ends:
        return disp[-30:]
    e = ends[-1]
    starts = [i for i, d in enumerate(disp[:e]) if d["kernel"].startswith("boost_update")]
    return disp[(starts[-1] if starts else max(0, e - 30)): e + 1]


def main():
    passes = [last_tree(load(p)) for p in sys.argv[1:]]
    n = min(len(p) for p in passes)
    merged = []
    for k in range(n):
        d = dict(passes[0][k])
        for p in passes[1:]:
            if p[k]["kernel"] != d["kernel"]:
                print(f"# dispatch {k}: kernel mismatch {p[k]['kernel'][:40]} vs {d['kernel'][:40]}")
            d.update({c: v for c, v in p[k].items() if c not in ("kernel", "grid")})
        merged.append(d)
    hdr = (f"{'#':>2s} {'kernel':44s} {'fetch MB':>9s} {'write MB':>9s} {'LDS confl':>9s} "
           f"{'LDS wait/inst':>13s} {'vs L0 fetch':>11s}")
    print(hdr)
    l0 = None
    level = 0
    for i, d in enumerate(merged):
        k = d["kernel"]
        fetch = d.get("FETCH_SIZE", 0.0) / 1024.0          # KB -> MB
        write = d.get("WRITE_SIZE", 0.0) / 1024.0
        act = d.get("SQ_LDS_IDX_ACTIVE", 0.0)
        conf = d.get("SQ_LDS_BANK_CONFLICT", 0.0) / act if act else float("nan")
        inst = d.get("SQ_INSTS_LDS", 0.0)
        wait = d.get("SQ_WAIT_INST_LDS", 0.0) / inst if inst else float("nan")
        rel = ""
        name = k.split("(")[0][:44]
        if k.startswith("hist_build"):
            if l0 is None:
                l0 = fetch
            rel = f"{fetch / l0:11.2f}" if l0 else ""
            name = f"L{level} {name}"[:44]
            level += 1
        print(f"{i:2d} {name:44s} {fetch:9.1f} {write:9.1f} {conf:9.1%} {wait:13.1f} {rel:>11s}")


if __name__ == "__main__":
    main()
