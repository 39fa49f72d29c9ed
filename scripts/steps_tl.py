"""Kernel timeline between two consecutive matrix writes (k_rows, k_rows_w or,
when every class is heavy, k_heavy_rows_t) of a
rocprofv3 kernel-trace CSV: every kernel from the start of write K-1 to the
end of write K, relative to write K-1's start, with its queue.
Usage: python scripts/steps_tl.py run_kernel_trace.csv [K]"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1]))
        if "elementwise" not in r["Kernel_Name"] and "FillFunctor" not in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
kr = [i for i, r in enumerate(rows)
      if any(w in r["Kernel_Name"] for w in ("k_rows<", "k_rows_w<", "k_heavy_rows_t"))]
if not any("k_rows" in rows[i]["Kernel_Name"] for i in kr):
    pass
else:
    kr = [i for i in kr if "k_heavy_rows_t" not in rows[i]["Kernel_Name"]]
k = int(sys.argv[2]) if len(sys.argv) > 2 else len(kr) - 2
a, b = kr[k - 1], kr[k]
t0 = int(rows[a]["Start_Timestamp"])
tend = int(rows[b]["End_Timestamp"])
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s < t0 or s > tend:
        continue
    print(f"{(s - t0) / 1000:8.1f} {(e - t0) / 1000:8.1f} {(e - s) / 1000:6.1f} q{r['Queue_Id']} "
          f"{r['Kernel_Name'][:52]}")
print(f"write-to-write {(int(rows[b]['Start_Timestamp']) - t0) / 1000:.1f} us")
