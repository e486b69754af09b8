#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace: top kernels + the dispatch timeline of
one boosting step (between two boost_update launches)."""
import csv
import glob
import sys

d = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "boost_update"   # kernel that starts a step
stats = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)
trace = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)
if stats:
    r = list(csv.DictReader(open(stats[0])))
    print("== top kernels ==")
    for x in r[:14]:
        print(f"{x['Name'][:64]:64s} calls={x['Calls']:>5s} avg={float(x['AverageNs'])/1e3:8.1f}us "
              f"tot={float(x['TotalDurationNs'])/1e6:8.2f}ms {float(x['Percentage']):5.1f}%")
if trace:
    t = sorted(csv.DictReader(open(trace[0])), key=lambda x: int(x["Start_Timestamp"]))
    bu = [i for i, x in enumerate(t) if marker in x["Kernel_Name"]]
    if len(bu) >= 3:
        a, b = bu[-2], bu[-1]
        t0 = int(t[a]["Start_Timestamp"])
        print(f"== one step: {(int(t[b]['Start_Timestamp']) - t0) / 1e3:.1f} us ==")
        busy = 0
        for x in t[a:b]:
            s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
            busy += e - s
            name = x["Kernel_Name"].split("(")[0][:44]
            print(f"  +{(s - t0) / 1e3:8.1f}us {(e - s) / 1e3:8.1f}us  {name}  grid={x['Grid_Size_X']}x{x['Grid_Size_Y']} "
                  f"wg={x['Workgroup_Size_X']} lds={x['LDS_Block_Size']} vgpr={x['VGPR_Count']}")
        print(f"  kernel-busy {busy / 1e3:.1f} us")
