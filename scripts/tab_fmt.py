"""Format the last bench line for scripts/tab.sh."""
import json
import os
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = d["step_ms"]
t = os.environ.get("T", "")
print(f"{t:<40} mean {d['ms_per_step']:.4f} min {s['min']:.4f} med {s['median']:.4f} "
      f"p90 {s['p90']:.4f} k_rows {d['roofline']['avg_launch_ms']:.4f}")
