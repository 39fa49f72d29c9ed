#!/bin/bash
# The bench line's placement field and k_rows time under several mprobe settings.
set -u
mkdir -p gpurun_out
for t in ${AB:-"mprobe=8"}; do
  KANO_TUNE="$t" timeout -k 10 150 python3 bench.py --steps ${STEPS:-300} --warmup 20 --cpu-baseline 0 > gpurun_out/pp.log 2>&1 || exit $?
  tail -1 gpurun_out/pp.log | T="$t" python3 -c "import json,os,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(os.environ['T'], 'k_rows', round(r['avg_launch_ms'],4), 'placement', r['placement']['candidates'], r['placement']['kept_probe_ms'], r['placement']['slowest_probe_ms'])"
done
