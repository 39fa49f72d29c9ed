#!/bin/bash
# rocprofv3 hip-trace + kernel-trace of a short C3 bench (EXTRA: more bench
# flags), merged into one host / GPU timeline of the last step.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/ht
timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace -d gpurun_out/ht -o run --output-format csv -- \
  python3 bench.py --steps 8 --warmup 3 --cpu-baseline 0 ${EXTRA:-} > gpurun_out/ht.log 2>&1 || exit $?
python3 scripts/host_timeline.py gpurun_out/ht > gpurun_out/host_timeline${TAG:-}.txt
echo done
