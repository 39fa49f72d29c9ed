#!/bin/bash
# C4 / C5 kernel profiles and a k_rows column-chunk sweep on C5.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for t in ${C5_TUNES:-"cww=8192" "cww=4096" "cww=2048"}; do
  KANO_TUNE="$t" timeout -k 10 400 python bench.py --config C5 --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/c5_tune.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "c5 $t rc=$rc"; tail -3 gpurun_out/c5_tune.log; exit $rc; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/c5_tune.log').read().strip().splitlines()[-1])
print('C5 $t', round(d['ms_per_step'],3), 'k_rows', round(d['roofline']['avg_launch_ms'],3), 'GB/s', round(d['roofline']['achieved']), d['stages_ms_last_step'])"
done
rm -rf gpurun_out/prof_c4 gpurun_out/prof_c5
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run --output-format csv -- python3 bench.py --config C4 --no-shadow --steps 3 --warmup 1 --cpu-baseline 0 > gpurun_out/prof_c4.log 2>&1
rc=$?; echo "prof c4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- python3 bench.py --config C5 --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/prof_c5.log 2>&1
rc=$?; echo "prof c5 rc=$rc"; exit $rc
