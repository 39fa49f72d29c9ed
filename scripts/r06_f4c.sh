#!/bin/bash
# the engine's 2 x 2 / KC = 8 fp4 GEMM: micro, MFMA parity tests, D1 lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./build_micro/gemm_f4 8000 8000 10000 0.05 20 > gpurun_out/gemm_f4.txt 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_path.py tests/test_gpu_parity.py -k "path or build_paths_agree or mfma or dense" > gpurun_out/f4c_tests.txt 2>&1 || exit 2
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_configs.py -k "D1" > gpurun_out/f4c_tests_d1.txt 2>&1 || exit 3
TUNES="-;hgemm=44" CFG="--config D1 --steps 30 --warmup 5" REPS=3 bash scripts/r06_tune_ab.sh > gpurun_out/f4c_ab.txt 2>&1 || exit 4
