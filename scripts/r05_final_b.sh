#!/bin/bash
# Round-5 final evidence, part B: D1 under rocprofv3 --kernel-trace --stats
# (kernel stats + the profiled line), and a C5 rank-0-of-8 step timeline.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/d1prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/d1prof -o run --output-format csv -- \
  python3 bench.py --config D1 --steps 20 --warmup 5 --cpu-baseline 0 --cold 0 > gpurun_out/d1prof.log 2>&1 || exit $?
grep "^{" gpurun_out/d1prof.log | tail -1 > gpurun_out/d1prof_line.json
python3 scripts/steps_tl.py gpurun_out/d1prof/run_kernel_trace.csv 12 > gpurun_out/d1_timeline_final.txt
bash scripts/c5r8_tl.sh > gpurun_out/c5r8_timeline_final.txt 2>&1 || exit $?
head -3 gpurun_out/c5r8_timeline_final.txt
