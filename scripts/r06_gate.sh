#!/bin/bash
# the gates' wait (engine-stream idle at the step boundary) on the C3 lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -k "pipelined" > gpurun_out/gate_tests.txt 2>&1 || exit 2
for cfg in "--steps 1000 --warmup 30" "--steps 400 --warmup 20 --rank-of 8"; do
  timeout -k 10 300 python bench.py --cpu-baseline 0 --cold 0 --alone 0 $cfg > gpurun_out/gate.json 2> gpurun_out/gate.err || exit 3
  python3 -c "
import json
d=json.loads(open('gpurun_out/gate.json').read().strip().splitlines()[-1])
print('$cfg', round(d['ms_per_step'],4), d['step_ms']['median'], d['verified'], d['boundary_idle_us'], d['host_us']['between_mean'])"
done
