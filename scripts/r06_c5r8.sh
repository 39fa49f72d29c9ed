#!/bin/bash
# C5 rank 0 of 8: the bench line and one step timeline (two writes)
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --config C5 --rank-of 8 --steps 20 --warmup 3 --cpu-baseline 0 --cold 0 --alone 2 ${EXTRA:-} > gpurun_out/c5r8.json 2>gpurun_out/c5r8.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/c5r8.err; exit $rc; }
python3 -c "
import json
d=json.loads(open('gpurun_out/c5r8.json').read().strip().splitlines()[-1])
print('step', d['ms_per_step'], d['step_ms']['median'], 'verified', d['verified'], 'write', d['roofline']['avg_launch_ms'], d['roofline']['frac'], 'alone', d['roofline']['alone'])"
rm -rf gpurun_out/c5tl
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/c5tl -o run --output-format csv -- \
  python3 bench.py --config C5 --rank-of 8 --steps 5 --warmup 2 --cpu-baseline 0 --cold 0 --alone 0 ${EXTRA:-} > gpurun_out/c5tl.log 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "tl rc=$rc"; tail -5 gpurun_out/c5tl.log; exit $rc; }
python3 scripts/steps_tl.py $(find gpurun_out/c5tl -name "*kernel_trace.csv" | head -1) > gpurun_out/c5r8_tl.txt
cat gpurun_out/c5r8_tl.txt
