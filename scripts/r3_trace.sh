#!/bin/bash
# Kernel (+ HIP API) trace of short bench runs, one per spec; prints the
# step timeline between two matrix writes (scripts/steps_tl.py).
#   SPECS="label|KANO_TUNE|bench args;label2|...|..."   HIPTR=1 adds --hip-trace
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
IFS=';' read -ra specs <<< "$SPECS"
for s in "${specs[@]}"; do
  IFS='|' read -r label tune args <<< "$s"
  rm -rf gpurun_out/tr_$label
  KANO_TUNE="$tune" timeout -k 10 200 rocprofv3 --kernel-trace ${HIPTR:+--hip-trace} --stats -d gpurun_out/tr_$label -o run \
    --output-format csv -- python3 bench.py --steps 20 --warmup 5 --cpu-baseline 0 $args > gpurun_out/tr_$label.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$label rc=$rc"; tail -5 gpurun_out/tr_$label.log; exit $rc; }
  f=$(find gpurun_out/tr_$label -name "*kernel_trace.csv" | head -1)
  echo "== $label ($tune) $args"
  python3 scripts/steps_tl.py "$f" > gpurun_out/tl_$label.txt && tail -60 gpurun_out/tl_$label.txt
  cp $(find gpurun_out/tr_$label -name "*kernel_stats.csv" | head -1) gpurun_out/ks_$label.csv
done
