#!/bin/bash
# the write on 3 whole XCDs with the engine streams on the other 5 (rxcd=3,
# emx=1) against the default on C3, rank 0 of 8, C4, D1, C5
set -u
: > gpurun_out/xcd_all.jsonl
for cfg in "--steps 600 --warmup 30" "--steps 400 --warmup 20 --rank-of 8" "--config C4 --steps 300 --warmup 20" "--config D1 --steps 30 --warmup 5" "--config C5 --steps 20 --warmup 3"; do
  TUNES="-;rxcd=3,emx=1" CFG="$cfg" REPS=2 bash scripts/r06_tune_ab.sh > /dev/null 2>&1 || exit 1
  sed "s|^{|{\"cfg\": \"$cfg\", |" gpurun_out/tune_ab.jsonl >> gpurun_out/xcd_all.jsonl
done
cat gpurun_out/xcd_all.jsonl
