#!/bin/bash
# Round-5 final evidence, part A: the GPU suite, smoke(), the driver's bench
# command, the same under rocprofv3 --kernel-trace --stats, FETCH/WRITE PMC.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/gpu_tests_final.log 2>&1; rc=$?; tail -2 gpurun_out/gpu_tests_final.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
bash scripts/r05_evidence.sh
