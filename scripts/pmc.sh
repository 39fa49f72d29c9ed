#!/bin/bash
# HBM traffic of the bench's kernels from PMC counters: FETCH_SIZE and
# WRITE_SIZE need separate passes on gfx950 (TCC slots), each a kernel-trace
# run of its own (no sys/runtime trace with --pmc).  Output:
# gpurun_out/pmc_{fetch,write}/..._counter_collection.csv, summarised by
# scripts/pmc_summary.py.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in FETCH_SIZE WRITE_SIZE; do
  d=gpurun_out/pmc_$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  rm -rf "$d"
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace -d "$d" -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --cpu-baseline 0 ${BENCH_ARGS:-} > "$d.log" 2>&1
  rc=$?; echo "pmc $c rc=$rc"
  case "$rc" in 0) ;; *) exit $rc ;; esac
done
python3 scripts/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write > gpurun_out/pmc_summary.json
cat gpurun_out/pmc_summary.json | head -c 1500
