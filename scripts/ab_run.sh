#!/bin/bash
# GPU iteration: selected GPU tests (PYK), bench A/B over KANO_TUNE settings
# (AB, space-separated), the kernel timeline of the default setting.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${PYK:-verify or rows}" > gpurun_out/pytest_q.log 2>&1
rc=$?; echo "pytest_rc=$rc"; tail -3 gpurun_out/pytest_q.log; [ $rc -eq 0 ] || exit $rc
STEPS=${STEPS:-600} WARMUP=30 bash scripts/bab.sh ${AB:-""} || exit $?
bash scripts/tl.sh ${NK:-30} "" > gpurun_out/tl_q.txt 2>&1 || exit $?
echo done
