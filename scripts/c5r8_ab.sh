#!/bin/bash
# C5 rank 0 of 8 (emulated) bench lines under KANO_TUNE settings, in turn
#   scripts/c5r8_ab.sh "t1" "t2" ...
set -u
for t in "$@"; do
  KANO_TUNE="$t" timeout -k 10 300 python3 bench.py --config C5 --rank-of 8 --steps 12 --warmup 3 \
    --cpu-baseline 0 --cold 0 --alone 0 > gpurun_out/c5ab.log 2>&1 || { echo "$t failed"; tail -5 gpurun_out/c5ab.log; exit 1; }
  grep "^{" gpurun_out/c5ab.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('[%s] step mean %.3f median %.3f k_rows %.3f frac %.3f verified %s' % ('$t', d['ms_per_step'], d['step_ms']['median'], r['avg_launch_ms'], r['frac'], d.get('verified')))"
done
