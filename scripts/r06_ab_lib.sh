#!/bin/bash
# A/B of two engine builds: libkano_hip_base.so (the last commit) against the
# working tree's libkano_hip.so, alternating, on CFGS (bench.py arguments,
# ';'-separated); first the parity subset PYT (pytest -k) on the new one
set -u
mkdir -p gpurun_out
if [ -n "${PYT:-}" ]; then
  timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_configs.py -k "$PYT" > gpurun_out/ab_t.log 2>&1
  rc=$?; echo "pytest_rc=$rc"; tail -2 gpurun_out/ab_t.log
  case $rc in 0) ;; *) exit $rc ;; esac
fi
: > gpurun_out/ab_lib.jsonl
IFS=';' read -ra CF <<< "${CFGS:---steps 300 --warmup 20}"
for rep in $(seq 1 ${REPS:-3}); do
  for lib in base new; do
    for cfg in "${CF[@]}"; do
      if [ $lib = base ]; then L=kubernetes-verification_amd/csrc/libkano_hip_base.so; else L=kubernetes-verification_amd/csrc/libkano_hip.so; fi
      KANO_HIP_LIB=$L timeout -k 10 200 python bench.py --cpu-baseline 0 --cold 0 --alone 0 $cfg > gpurun_out/ab.json 2>gpurun_out/ab.err
      rc=$?; case $rc in 0) ;; *) echo "$lib $cfg rc=$rc"; tail -5 gpurun_out/ab.err; exit $rc ;; esac
      python3 -c "
import json
d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1])
print(json.dumps({'lib':'$lib','cfg':'$cfg','mean':round(d['ms_per_step'],4),'median':d['step_ms']['median'],'verified':d['verified'],'rows_ms':round(d['roofline']['avg_launch_ms'],4)}))" >> gpurun_out/ab_lib.jsonl
    done
  done
done
cat gpurun_out/ab_lib.jsonl
