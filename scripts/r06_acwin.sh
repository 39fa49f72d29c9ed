#!/bin/bash
# AC rows in LDS windows: parity (forced small windows, C5 full size), then
# the C5 / C5 rank 0 of 8 / C3 lines against the last commit's library
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_configs.py -k "rows_variants_forced or c5_full or C3 or C4 or D1" > gpurun_out/acwin_tests.txt 2>&1 || exit 2
PYT= CFGS="--config C5 --steps 20 --warmup 3;--config C5 --rank-of 8 --steps 20 --warmup 3;--steps 600 --warmup 30" REPS=2 bash scripts/r06_ab_lib.sh > gpurun_out/acwin_ab.txt 2>&1 || exit 3
