"""Print the kernel timeline of the last bench step from a rocprofv3
kernel-trace CSV (start/end relative to the window's first kernel, gap to
the previous kernel, queue).
Usage: python scripts/timeline.py gpurun_out/prof/run_kernel_trace.csv [nkernels]"""
import csv
import sys

path = sys.argv[1]
nk = int(sys.argv[2]) if len(sys.argv) > 2 else 48
rows = [r for r in csv.DictReader(open(path)) if "elementwise" not in r["Kernel_Name"]
        and "FillFunctor" not in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = rows[-nk:]
t0 = int(last[0]["Start_Timestamp"])
prev_end = t0
busy = 0
for r in last:
    s = int(r["Start_Timestamp"]) - t0
    e = int(r["End_Timestamp"]) - t0
    gap = s - (prev_end - t0)
    prev_end = max(prev_end, e + t0)
    busy += e - s
    print(f"{s / 1000:8.1f} {e / 1000:8.1f} {(e - s) / 1000:6.1f} gap{gap / 1000:6.1f} "
          f"q{r['Queue_Id']} {r['Kernel_Name'][:48]:48s} g={r['Grid_Size_X']}x{r['Grid_Size_Y']} "
          f"wg={r['Workgroup_Size_X']}")
print(f"span {(prev_end - t0) / 1000:.1f} us, kernel busy {busy / 1000:.1f} us")
