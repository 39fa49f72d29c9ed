#!/bin/bash
# the sort window default (sww 768 -> 256): parity subset, then C5 / C5 rank 0
# of 8 / C4 / C3 against the last commit's library
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_configs.py -k "rows_variants_forced or c5_full or C4 or C3" > gpurun_out/sww_tests.txt 2>&1 || exit 2
PYT= CFGS="--config C5 --steps 20 --warmup 3;--config C5 --rank-of 8 --steps 20 --warmup 3;--config C4 --steps 300 --warmup 20;--steps 600 --warmup 30" REPS=2 bash scripts/r06_ab_lib.sh > gpurun_out/sww_ab.txt 2>&1 || exit 3
