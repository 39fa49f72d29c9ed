#!/bin/bash
# the pipelined prologue: its parity test, then C3 / rank 0 of 8 with and
# without it (alternating, 300 steps each)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py -k "pipelined or async_completion or small_shapes" > gpurun_out/r06_pipe_t.log 2>&1
rc=$?; echo "pytest_rc=$rc"; tail -3 gpurun_out/r06_pipe_t.log
case $rc in 0) ;; *) exit $rc ;; esac
: > gpurun_out/r06_pipe_ab.jsonl
for rep in 1 2; do
  for p in 1 0; do
    for extra in "" "--rank-of 8"; do
      timeout -k 10 120 python bench.py --steps 300 --warmup 20 --cpu-baseline 0 --cold 0 --alone 2 --pipeline $p $extra > gpurun_out/ab.json 2>gpurun_out/ab.err
      rc=$?; echo "p=$p extra=$extra rc=$rc"; case $rc in 0) ;; *) tail -5 gpurun_out/ab.err; exit $rc ;; esac
      python3 -c "
import json,sys
d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1])
o={'pipe':$p,'extra':'$extra','mean':d['ms_per_step'],'median':d['step_ms']['median'],'verified':d['verified'],'krows':d['roofline']['avg_launch_ms'],'frac':d['roofline']['frac'],'host':d['host_us']}
print(json.dumps(o))" >> gpurun_out/r06_pipe_ab.jsonl
    done
  done
done
cat gpurun_out/r06_pipe_ab.jsonl | cut -c1-220
