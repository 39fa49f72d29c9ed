#!/bin/bash
# C5 rank 0 of 8 (emulated): the bench line and a kernel timeline of one step
#   scripts/c5r8_tl.sh [KANO_TUNE]
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/c5tl
KANO_TUNE="${1:-}" timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/c5tl -o run \
  --output-format csv -- python3 bench.py --config C5 --rank-of 8 --steps 8 --warmup 3 \
  --cpu-baseline 0 --cold 0 --alone 3 > gpurun_out/c5tl.log 2>&1
rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -5 gpurun_out/c5tl.log; exit $rc; }
grep "^{" gpurun_out/c5tl.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('step', d['ms_per_step'], d['step_ms']['median'], 'k_rows', r['avg_launch_ms'], r['frac'], 'alone', r.get('alone'))"
python3 scripts/steps_tl.py $(find gpurun_out/c5tl -name "*kernel_trace.csv" | head -1) ${K:-6}
