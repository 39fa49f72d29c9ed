#!/bin/bash
# Emulated rank-0-of-N step (bench.py --rank-of N) timings and one kernel
# timeline per N: what stays replicated when the rows shard.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for N in ${NS:-1 2 4 8}; do
  timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --cpu-baseline 0 --rank-of $N \
    --config ${CFG:-C3} > gpurun_out/rank_$N.log 2>&1 || exit $?
  python3 -c "
import json
for l in open('gpurun_out/rank_$N.log'):
    if l.startswith('{'):
        d=json.loads(l); print('N=$N', 'step', round(d['ms_per_step'],4), 'median', d['step_ms']['median'], 'k_rows', round(d['roofline']['avg_launch_ms'],4))"
done
rm -rf gpurun_out/rtl
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/rtl -o run --output-format csv -- \
  python3 bench.py --steps 6 --warmup 2 --cpu-baseline 0 --rank-of ${TLN:-8} --config ${CFG:-C3} \
  > gpurun_out/rtl.log 2>&1 || exit $?
python3 scripts/timeline.py $(find gpurun_out/rtl -name "*kernel_trace.csv" | head -1) 40
