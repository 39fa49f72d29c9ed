#!/bin/bash
# What the box's CPU controller does to the bench: cgroup quota and
# throttling counters around the driver's exact command.
set -u
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
echo "nproc $(nproc)  affinity $(python3 -c 'import os; print(len(os.sched_getaffinity(0)))')"
cg=$(awk -F: '$1=="0"{print $3}' /proc/self/cgroup)
echo "cgroup $cg"
for f in cpu.max cpu.weight cpu.stat cpuset.cpus.effective; do
  [ -r "/sys/fs/cgroup$cg/$f" ] && echo "$f: $(tr '\n' ' ' < /sys/fs/cgroup$cg/$f)"
done
for k in 1 2 3 4 5 6 7 8; do
  s0=$(cat /sys/fs/cgroup$cg/cpu.stat 2>/dev/null | tr '\n' ' ')
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/cp_$k.json 2>/dev/null || exit 1
  s1=$(cat /sys/fs/cgroup$cg/cpu.stat 2>/dev/null | tr '\n' ' ')
  python3 - "$k" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/cp_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print("run", sys.argv[1], round(d["ms_per_step"], 4), "max", d["step_ms"]["max"], d["host_us"])
PY
  echo "  before: $s0"
  echo "  after:  $s1"
done
