#!/bin/bash
# Quick GPU iteration: selected GPU tests (PYK), the default bench line, and
# the kernel timeline of the last steps (scripts/tl.sh).
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${PYK:-verify}" > gpurun_out/pytest_q.log 2>&1
rc=$?; echo "pytest_rc=$rc"; tail -3 gpurun_out/pytest_q.log; [ $rc -eq 0 ] || exit $rc
for t in ${TUNES:-""}; do :; done
KANO_TUNE="${TUNE:-}" timeout -k 10 200 python3 bench.py --cpu-baseline 0 ${BENCH_ARGS:-} > gpurun_out/bench_q.log 2>&1 || exit $?
tail -1 gpurun_out/bench_q.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('step', d['ms_per_step'], d['step_ms']['median'], 'k_rows', d['roofline']['avg_launch_ms'], d['roofline']['frac'], 'verified', d['verified'])"
KANO_TUNE="${TUNE:-}" bash scripts/tl.sh ${NK:-60} "${TUNE:-}" > gpurun_out/tl_q.txt 2>&1 || exit $?
echo done
