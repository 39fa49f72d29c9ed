"""Host API time per engine call from a rocprofv3 --hip-trace run: for the
last K calls of kano_verify / kano_verify_gather (delimited by the matrix
write's hipExtLaunchKernel), the count and total time of each HIP API
function and the host time outside HIP calls.
Usage: python scripts/api_breakdown.py DIR [K]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
K = int(sys.argv[2]) if len(sys.argv) > 2 else 10
api = sorted(csv.DictReader(open(glob.glob(d + "/*hip_api_trace.csv")[0])),
             key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(api) if r["Function"] == "hipExtLaunchKernel"]
if len(marks) < K + 1:
    K = len(marks) - 1
tot = collections.Counter()
cnt = collections.Counter()
outside = 0.0
span = 0.0
for a, b in zip(marks[-K - 1:-1], marks[-K:]):
    seg = api[a + 1:b + 1]
    t0 = int(api[a]["End_Timestamp"])
    t1 = int(api[b]["End_Timestamp"])
    span += (t1 - t0) / 1e3
    busy = 0.0
    for r in seg:
        du = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot[r["Function"]] += du
        cnt[r["Function"]] += 1
        busy += du
    outside += (t1 - t0) / 1e3 - busy
print(f"per call over {K} calls: span {span / K:.1f} us, outside HIP calls {outside / K:.1f} us")
for f, t in tot.most_common():
    print(f"  {f:32s} {cnt[f] / K:6.1f} calls  {t / K:8.1f} us  ({t / cnt[f]:.2f} us each)")
