"""Print the kernel timeline of the last few steps of a rocprofv3 kernel trace.
Usage: prof_steps.py OUTDIR [N_KERNELS] [SKIP_LAST]"""
import csv
import glob
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0
f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
r = sorted(csv.DictReader(open(f)), key=lambda x: int(x["Start_Timestamp"]))
if skip:
    r = r[:-skip]
r = r[-n:]
t0 = int(r[0]["Start_Timestamp"])
prev = None
busy = 0
for x in r:
    s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    prev = e
    busy += e - s
    print(f"{(s - t0) / 1e3:9.1f} gap {gap:6.1f} dur {(e - s) / 1e3:7.1f}  {x['Kernel_Name'][:58]:58s} "
          f"grid={x['Grid_Size_X']}x{x['Grid_Size_Y']}x{x['Grid_Size_Z']} wg={x['Workgroup_Size_X']}")
print(f"span {(prev - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us over {len(r)} kernels")
