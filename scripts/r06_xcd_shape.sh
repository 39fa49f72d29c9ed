#!/bin/bash
# the XCD split's shape: the build's streams unmasked (xcde=0) or sharing one
# XCD with the write (xcde=2), the write on 4 XCDs (xcdw=4) or 2 with the
# build on 6 (xcdw=2), against the default (write on XCDs 0-2, build on 3-7)
set -u
: > gpurun_out/xcd_shape.jsonl
for cfg in "--steps 600 --warmup 30" "--config C4 --steps 300 --warmup 20"; do
  TUNES="-;xcde=0;xcde=2;xcdw=4;xcdw=2" CFG="$cfg" REPS=2 bash scripts/r06_tune_ab.sh > /dev/null 2>&1 || exit 1
  sed "s|^{|{\"cfg\": \"$cfg\", |" gpurun_out/tune_ab.jsonl >> gpurun_out/xcd_shape.jsonl
done
cat gpurun_out/xcd_shape.jsonl
