#!/bin/bash
# k_rows tuning sweep: bench under several KANO_TUNE settings (C3).
set -u
mkdir -p gpurun_out
for t in ${TUNES:-"ch=16,align=16" "ch=24,align=16" "ch=16,align=32"}; do
  KANO_TUNE="$t" timeout -k 10 200 python bench.py --steps 20 --cpu-baseline 0 ${BENCH_ARGS:-} > gpurun_out/tune.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "tune $t rc=$rc"; tail -5 gpurun_out/tune.log; exit $rc; fi
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/tune.log').read().strip().splitlines()[-1])
print('$t', round(d['ms_per_step'],4), d['step_ms'], 'k_rows', round(d['roofline']['avg_launch_ms'],4), 'GB/s', round(d['roofline']['achieved']))"
done
