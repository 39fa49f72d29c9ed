#!/bin/bash
# The round's evidence in one GPU call: parity tests, smoke, the default
# bench line (with cpu_baseline), its rocprofv3 kernel-trace --stats profile,
# and the FETCH_SIZE / WRITE_SIZE PMC passes (scripts/pmc.sh).
set -u
mkdir -p gpurun_out
bash scripts/gpu_check.sh || exit $?
bash scripts/pmc.sh || exit $?
