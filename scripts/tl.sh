#!/bin/bash
# Kernel timeline of the last bench step under each KANO_TUNE setting:
#   tl.sh NKERNELS "t1" "t2" ...        (CFG from the env)
set -u
nk=$1; shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for t in "$@"; do
  rm -rf gpurun_out/tl
  KANO_TUNE="$t" timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/tl -o run \
    --output-format csv -- python3 bench.py --steps 6 --warmup 2 --cpu-baseline 0 \
    --config ${CFG:-C3} ${EXTRA:-} > gpurun_out/tl.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$t rc=$rc"; tail -5 gpurun_out/tl.log; exit $rc; }
  echo "== $t"
  python3 scripts/timeline.py $(find gpurun_out/tl -name "*kernel_trace.csv" | head -1) $nk
done
