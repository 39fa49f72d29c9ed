#!/bin/bash
# Emulated per-rank steps (rank 0 of N on one GPU) and the C4 / C5 lines.
set -u
mkdir -p gpurun_out
for N in 2 4 8; do
  timeout -k 10 200 python3 bench.py --rank-of $N --steps ${STEPS:-600} --warmup 30 --cpu-baseline 0 > gpurun_out/rank_of_$N.log 2>&1 || exit $?
  tail -1 gpurun_out/rank_of_$N.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('rank-of-$N step', round(d['ms_per_step'],4), 'median', d['step_ms']['median'], 'k_rows', round(d['roofline']['avg_launch_ms'],4))"
done
for C in C4 C5; do
  timeout -k 10 300 python3 bench.py --config $C --steps ${STEPS5:-100} --warmup 5 --cpu-baseline 0 > gpurun_out/bench_$C.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_$C.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$C step', round(d['ms_per_step'],4), 'median', d['step_ms']['median'], 'k_rows', round(d['roofline']['avg_launch_ms'],4), 'frac', round(d['roofline']['frac'],3), 'verified', d['verified'])"
done
echo done
