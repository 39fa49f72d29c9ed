#!/bin/bash
# the every-XCD masked side stream (its own queue) where the XCD split does
# not apply (sideu=1): rank 0 of 2 and 8, D1, C5 rank 0 of 8
set -u
timeout -k 10 300 env KANO_TUNE=sideu=1 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "pipelined" > gpurun_out/sideu_tests.txt 2>&1 || { tail -20 gpurun_out/sideu_tests.txt; exit 1; }
tail -1 gpurun_out/sideu_tests.txt
: > gpurun_out/sideu.jsonl
for cfg in "--steps 400 --warmup 20 --rank-of 2" "--steps 400 --warmup 20 --rank-of 8" "--config D1 --steps 30 --warmup 5" "--config C5 --rank-of 8 --steps 20 --warmup 3"; do
  TUNES="-;sideu=1" CFG="$cfg" REPS=2 bash scripts/r06_tune_ab.sh > /dev/null 2>&1 || exit 1
  sed "s|^{|{\"cfg\": \"$cfg\", |" gpurun_out/tune_ab.jsonl >> gpurun_out/sideu.jsonl
done
cat gpurun_out/sideu.jsonl
