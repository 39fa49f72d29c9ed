#!/bin/bash
# the fused one-rank list pass (k_verify_cols_f) against the count scan +
# k_idx_write form on C4, D1, C5
set -u
: > gpurun_out/vf_all.jsonl
for cfg in "--config C4 --steps 300 --warmup 20" "--config D1 --steps 30 --warmup 5" "--config C5 --steps 20 --warmup 3"; do
  TUNES="-;vfused=0" CFG="$cfg" REPS=2 bash scripts/r06_tune_ab.sh > /dev/null 2>&1 || exit 1
  sed "s|^{|{\"cfg\": \"$cfg\", |" gpurun_out/tune_ab.jsonl >> gpurun_out/vf_all.jsonl
done
cat gpurun_out/vf_all.jsonl
