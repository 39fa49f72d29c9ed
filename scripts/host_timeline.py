"""Merged host-API / kernel timeline of the last bench step from a rocprofv3
--hip-trace --kernel-trace run (round 2): shows where the host's issue, not
the GPU, sets the pace.
Usage: python scripts/host_timeline.py DIR   (DIR holds run_hip_api_trace.csv
and run_kernel_trace.csv)"""
import csv
import glob
import sys

d = sys.argv[1]
api = sorted(csv.DictReader(open(glob.glob(d + "/*hip_api_trace.csv")[0])),
             key=lambda r: int(r["Start_Timestamp"]))
ker = sorted(csv.DictReader(open(glob.glob(d + "/*kernel_trace.csv")[0])),
             key=lambda r: int(r["Start_Timestamp"]))
rows = [k for k in ker if "k_rows" in k["Kernel_Name"]]
t0 = int(rows[-2]["End_Timestamp"])          # from the second-to-last matrix write's end
t1 = int(rows[-1]["End_Timestamp"])
ev = []
for r in api:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if t0 <= s <= t1 and r["Function"] not in ("hipGetLastError",):
        ev.append((s, e, "host", r["Function"]))
for k in ker:
    s, e = int(k["Start_Timestamp"]), int(k["End_Timestamp"])
    if t0 - 5000 <= s <= t1:
        ev.append((s, e, "gpu q%s" % k["Queue_Id"], k["Kernel_Name"].split("(")[0][:44]))
ev.sort()
for s, e, w, n in ev:
    print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:6.1f}  {w:8s} {n}")
