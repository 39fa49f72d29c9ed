#!/bin/bash
# Round 6: the fp4 GEMM -- micro (i8 vs fp4 forms), the MFMA parity tests,
# and D1's bench line (base library vs the working tree's when present)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./build_micro/gemm_f4 8000 8000 10000 0.05 20 > gpurun_out/gemm_f4.txt 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -k "build_paths_agree or mfma or dense" > gpurun_out/f4_tests.txt 2>&1 || exit 2
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_configs.py -k "D1 or C4 or dense or mfma" > gpurun_out/f4_tests_cfg.txt 2>&1 || exit 3
for rep in 1 2; do
  for lib in base work; do
    if [ $lib = base ]; then export KANO_HIP_LIB=$PWD/kubernetes-verification_amd/csrc/libkano_hip_base.so; else unset KANO_HIP_LIB; fi
    timeout -k 10 300 python bench.py --config D1 --steps 30 --warmup 5 --cpu-baseline 0 --cold 0 \
      > gpurun_out/d1_${lib}_${rep}.json 2> gpurun_out/d1_${lib}_${rep}.err || exit 4
  done
done
python3 - <<'PY'
import json
for rep in (1, 2):
    for lib in ("base", "work"):
        d = json.loads(open(f"gpurun_out/d1_{lib}_{rep}.json").read().strip().splitlines()[-1])
        m = d.get("mfma_roofline") or {}
        print(lib, rep, "step median", d["step_ms"]["median"], "mean", round(d["ms_per_step"], 4),
              "gemm ms", round(m.get("avg_ms", 0), 4), "achieved", round(m.get("achieved", 0)),
              "alone", m.get("alone"), "verified", d.get("verified"))
PY
