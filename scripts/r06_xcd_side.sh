#!/bin/bash
# the side stream's XCDs under the split: automatic (default: every XCD unless
# the last build had heavy classes), always on every XCD (xcdside=0), always with
# the engine stream on XCDs 3-7 (xcdside=1); C3, C4, and the parity test
set -u
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "pipelined" > gpurun_out/xcd_side_tests.txt 2>&1 || { tail -20 gpurun_out/xcd_side_tests.txt; exit 1; }
tail -2 gpurun_out/xcd_side_tests.txt
: > gpurun_out/xcd_side.jsonl
for cfg in "--steps 600 --warmup 30" "--config C4 --steps 300 --warmup 20"; do
  TUNES="-;xcdside=0;xcdside=1" CFG="$cfg" REPS=2 bash scripts/r06_tune_ab.sh > /dev/null 2>&1 || exit 1
  sed "s|^{|{\"cfg\": \"$cfg\", |" gpurun_out/tune_ab.jsonl >> gpurun_out/xcd_side.jsonl
done
cat gpurun_out/xcd_side.jsonl
