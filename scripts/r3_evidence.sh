#!/bin/bash
# Round-3 evidence: the PMC traffic passes (pmc.sh), the driver's command
# repeated plus one --hip-trace run of it (r3_b20x.sh), and the emulated
# rank-0-of-N steps.  Every step bounded; stops at the first failure.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash scripts/pmc.sh > gpurun_out/pmc.out 2>&1 || { tail -5 gpurun_out/pmc.out; exit 1; }
tail -c 600 gpurun_out/pmc.out; echo
REPS="1 2 3" TRACE=1 bash scripts/r3_b20x.sh || exit 1
for N in ${RANKS:-2 4 8}; do
  timeout -k 10 200 python3 bench.py --steps 300 --warmup 20 --rank-of $N --cpu-baseline 0 \
      > gpurun_out/rank_of_$N.json 2> gpurun_out/rank_of_$N.err || { tail gpurun_out/rank_of_$N.err; exit 1; }
  python3 - "$N" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/rank_of_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print("rank_of", sys.argv[1], "ms", round(d["ms_per_step"], 4), "median", d["step_ms"]["median"],
      "k_rows", round(d["roofline"]["avg_launch_ms"], 4), "cus", d["roofline"].get("cus"))
PY
done
