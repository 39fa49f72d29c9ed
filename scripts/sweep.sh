#!/bin/bash
# bench under several KANO_TUNE settings:  sweep.sh CONFIG STEPS "t1" "t2" ...
set -u
cfg=$1; steps=$2; shift 2
mkdir -p gpurun_out
extra=""
[ "$cfg" = "C4" ] && extra="--no-shadow"
for t in "$@"; do
  KANO_TUNE="$t" timeout -k 10 400 python bench.py --config $cfg --steps $steps --warmup ${WARMUP:-1} --cpu-baseline 0 $extra ${EXTRA:-} > gpurun_out/sweep.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "$cfg $t rc=$rc"; tail -5 gpurun_out/sweep.log; exit $rc; fi
  python3 -c "
import json; d=json.loads(open('gpurun_out/sweep.log').read().strip().splitlines()[-1])
print('$cfg', '$t', round(d['ms_per_step'],4), d['step_ms']['median'], 'k_rows', round(d['roofline']['avg_launch_ms'],4), 'GB/s', round(d['roofline']['achieved']), 'worst', d['step_ms'].get('worst5'), d['step_ms'].get('worst5_at'))"
done
