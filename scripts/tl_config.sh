#!/bin/bash
# a bench config's kernel timeline (one step between two matrix writes)
#   scripts/tl_config.sh CONFIG [KANO_TUNE] [bench args...]
set -u
CFG=$1; TUNE="${2:-}"; shift; shift || true
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/tlc
KANO_TUNE="$TUNE" timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tlc -o run --output-format csv -- \
  python3 bench.py --config "$CFG" --steps 12 --warmup 4 --cpu-baseline 0 --cold 0 --alone 0 "$@" > gpurun_out/tlc.log 2>&1 || exit $?
python3 scripts/steps_tl.py gpurun_out/tlc/run_kernel_trace.csv 10 > gpurun_out/tl_$CFG.txt
head -60 gpurun_out/tl_$CFG.txt
