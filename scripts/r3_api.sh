#!/bin/bash
# rocprofv3 --hip-trace of short bench runs, the host API time per call
# (scripts/api_breakdown.py).  SPECS="label|KANO_TUNE|bench args;..."
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
IFS=';' read -ra specs <<< "$SPECS"
for s in "${specs[@]}"; do
  IFS='|' read -r label tune args <<< "$s"
  rm -rf gpurun_out/api_$label
  KANO_TUNE="$tune" timeout -k 10 200 rocprofv3 --hip-trace -d gpurun_out/api_$label -o run \
    --output-format csv -- python3 bench.py --steps 30 --warmup 5 --cpu-baseline 0 $args > gpurun_out/api_$label.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$label rc=$rc"; tail -5 gpurun_out/api_$label.log; exit $rc; }
  echo "== $label ($tune) $args"
  python3 scripts/api_breakdown.py gpurun_out/api_$label 20 | tee gpurun_out/api_$label.txt
  rm -rf gpurun_out/api_$label
done
