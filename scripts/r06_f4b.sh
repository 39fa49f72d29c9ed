#!/bin/bash
# fp4 contraction follow-up: GEMM micro (tile / chunk variants), the path and
# MFMA parity tests, the path bench (fp4 k_path_mfma)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./build_micro/gemm_f4 8000 8000 10000 0.05 20 > gpurun_out/gemm_f4.txt 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_path.py tests/test_gpu_parity.py -k "path or build_paths_agree or mfma or dense" > gpurun_out/f4b_tests.txt 2>&1 || exit 2
timeout -k 10 300 python scripts/path_bench.py --config C3 > gpurun_out/path_bench_c3.txt 2>&1 || exit 3
