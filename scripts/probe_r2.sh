#!/bin/bash
# Round-2 probe: the store-shape micro, the engine's host timing of the bench
# step, and a hip-trace of a short bench (host API costs per step).
set -u
mkdir -p gpurun_out
timeout -k 10 120 scripts/micro/store_bw2 > gpurun_out/store_bw2.txt 2>&1 || exit $?
KANO_TUNE=hosttime=1 timeout -k 10 200 python3 bench.py --steps 1000 --warmup 50 --cpu-baseline 0 > gpurun_out/hosttime.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace -d gpurun_out/ht -o run --output-format csv -- \
  python3 bench.py --steps 6 --warmup 2 --cpu-baseline 0 > gpurun_out/ht.log 2>&1 || exit $?
echo done
