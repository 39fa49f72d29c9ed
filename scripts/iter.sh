#!/bin/bash
# One GPU iteration: parity tests, a KANO_TUNE sweep (args), and a kernel-trace
# profile of the default bench with the top kernels printed.
#   iter.sh "t1" "t2" ...      (CFG, STEPS, EXTRA, PROF_ARGS from the env)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^(E |FAILED)" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
if [ $# -gt 0 ]; then
  WARMUP=5 bash scripts/sweep.sh ${CFG:-C3} ${STEPS:-100} "$@" || exit $?
fi
if [ "${PROFILE:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  rm -rf gpurun_out/prof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv \
    -- python3 bench.py --steps 5 --warmup 2 --cpu-baseline 0 --config ${CFG:-C3} ${PROF_ARGS:-} \
    > gpurun_out/prof.log 2>&1
  rc=$?; echo "prof_rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 - <<'EOF'
import csv, glob
f = glob.glob("gpurun_out/prof/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in rows[:24]:
    print(f"{float(r['AverageNs'])/1000:8.1f} us x{r['Calls']:>3}  {r['Name'][:70]}")
EOF
fi
