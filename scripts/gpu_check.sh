#!/bin/bash
# One GPU session: parity tests, smoke, bench, kernel-trace profile.
# Each GPU step has its own time limit; a crash / timeout / abort ends the
# script (no further GPU step in the same call).
set -u
mkdir -p gpurun_out
stop_if_fatal() {  # $1 = exit code of a GPU step
  case "$1" in 0|1) return 0 ;; *) echo "fatal rc=$1, stopping"; exit "$1" ;; esac
}
timeout -k 10 ${T_TEST:-900} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest_rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; stop_if_fatal $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke_rc=$rc"; tail -2 gpurun_out/smoke.log; stop_if_fatal $rc
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench_rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-600; stop_if_fatal $rc
if [ "${PROFILE:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 50 --warmup 2 --cpu-baseline 0 ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1
  rc=$?; echo "prof_rc=$rc"; stop_if_fatal $rc
  find gpurun_out/prof -name "*stats*" | head
fi
