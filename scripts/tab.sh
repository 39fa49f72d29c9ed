#!/bin/bash
# Step-time A/B of the bench under KANO_TUNE settings (no profiler):
#   tab.sh "t1" "t2" ...      (CFG, EXTRA, REPS from the env)
set -u
mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
for t in "$@"; do
  KANO_TUNE="$t" timeout -k 10 120 python3 bench.py --steps ${STEPS:-50} --warmup 5 --cpu-baseline 0 \
    --config ${CFG:-C3} ${EXTRA:-} > gpurun_out/tab.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$t rc=$rc"; tail -5 gpurun_out/tab.log; exit $rc; }
  T="$t" python3 scripts/tab_fmt.py gpurun_out/tab.log
done
done
