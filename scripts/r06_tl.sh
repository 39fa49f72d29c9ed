#!/bin/bash
# step timelines (two consecutive matrix writes) with / without the pipelined
# prologue: CFG, EXTRA from the env
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for p in ${PIPES:-1 0}; do
  rm -rf gpurun_out/tl$p
  timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/tl$p -o run --output-format csv -- \
    python3 bench.py --steps ${STEPS:-8} --warmup 2 --cpu-baseline 0 --cold 0 --alone 0 \
    --pipeline $p --config ${CFG:-C3} ${EXTRA:-} > gpurun_out/tl$p.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "p=$p rc=$rc"; tail -5 gpurun_out/tl$p.log; exit $rc; }
  echo "== pipeline $p"
  python3 scripts/steps_tl.py $(find gpurun_out/tl$p -name "*kernel_trace.csv" | head -1) > gpurun_out/tl$p.txt
  cat gpurun_out/tl$p.txt
done
