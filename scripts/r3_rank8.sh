#!/bin/bash
# The emulated rank 0 of 8 (bench.py --rank-of 8) under knob variants, then
# one kernel trace of it.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for t in ${AB:-none rcu=0 async=0}; do
  KANO_TUNE="$t" timeout -k 10 200 python3 bench.py --steps 300 --warmup 20 --rank-of ${N:-8} --cpu-baseline 0 \
      > gpurun_out/r8.json 2> gpurun_out/r8.err || { tail gpurun_out/r8.err; exit 1; }
  python3 - "$t" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/r8.json").read().strip().splitlines()[-1])
print("r8", sys.argv[1], "ms", round(d["ms_per_step"], 4), "median", d["step_ms"]["median"],
      "k_rows", round(d["roofline"]["avg_launch_ms"], 4), "cus", d["roofline"].get("cus"), d["host_us"])
PY
done
rm -rf gpurun_out/r8tr
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r8tr -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --rank-of ${N:-8} --cpu-baseline 0 > gpurun_out/r8tr.log 2>&1 || exit $?
echo traced
