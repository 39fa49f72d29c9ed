#!/bin/bash
# Host time per call at rank 0 of 8 (emulated) and at N=1 (engine hosttime knob).
set -u
mkdir -p gpurun_out
for a in "--rank-of 8" ""; do
  KANO_TUNE=hosttime=1 timeout -k 10 150 python3 bench.py --steps 600 --warmup 30 --cpu-baseline 0 $a > gpurun_out/ht8.log 2>&1 || exit $?
  echo "== ${a:-N=1}"; grep "kano host" gpurun_out/ht8.log
  tail -1 gpurun_out/ht8.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('step', round(d['ms_per_step'],4), 'median', d['step_ms']['median'], 'k_rows', round(d['roofline']['avg_launch_ms'],4))"
done
