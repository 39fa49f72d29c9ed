#!/bin/bash
# rocprofv3 kernel stats of the driver's bench command (the profiled run's own
# line kept beside them), then the PMC traffic passes.  Bounded steps; stops
# at the first failure.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/kstats
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kstats -o run --output-format csv -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline 0 --cold 0 --alone 0 > gpurun_out/kstats.json 2> gpurun_out/kstats.err || { tail gpurun_out/kstats.err; exit 1; }
cp $(find gpurun_out/kstats -name "*kernel_stats.csv" | head -1) gpurun_out/kstats_c3.csv
python3 scripts/steps_tl.py $(find gpurun_out/kstats -name "*kernel_trace.csv" | head -1) > gpurun_out/kstats_tl.txt
rm -rf gpurun_out/kstats
head -6 gpurun_out/kstats_c3.csv | cut -c1-160
BENCH_ARGS="--alone 0 --cold 0" bash scripts/pmc.sh > gpurun_out/pmc.out 2>&1 || { tail -5 gpurun_out/pmc.out; exit 1; }
tail -c 800 gpurun_out/pmc.out; echo
