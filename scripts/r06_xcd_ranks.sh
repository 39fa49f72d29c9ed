#!/bin/bash
# the XCD split (with the side stream's placement rule) at the rank-0-of-2 / 4
# shard sizes (0.63 / 0.31 GB writes) via xcdmin, against the 1 GiB default
set -u
: > gpurun_out/xcd_ranks.jsonl
for cfg in "--steps 400 --warmup 20 --rank-of 2" "--steps 400 --warmup 20 --rank-of 4"; do
  TUNES="-;xcdmin=0" CFG="$cfg" REPS=3 bash scripts/r06_tune_ab.sh > /dev/null 2>&1 || exit 1
  sed "s|^{|{\"cfg\": \"$cfg\", |" gpurun_out/tune_ab.jsonl >> gpurun_out/xcd_ranks.jsonl
done
cat gpurun_out/xcd_ranks.jsonl
