#!/bin/bash
# rocprofv3 kernel stats of the bench under each KANO_TUNE setting; prints the
# average of the kernels matching $PAT (default: all front-end kernels)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for t in "$@"; do
  rm -rf gpurun_out/ks
  KANO_TUNE="$t" timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ks -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --cpu-baseline 0 --config ${CFG:-C3} > gpurun_out/ks.log 2>&1 || exit $?
  echo "== ${t:-(default)}"
  f=$(find gpurun_out/ks -name "*kernel_stats.csv" | head -1)
  python3 - "$f" "${PAT:-.}" <<'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    if re.search(sys.argv[2], r["Name"]) and "elementwise" not in r["Name"]:
        print(f'{float(r["AverageNs"])/1e3:8.1f} us  x{r["Calls"]:>4}  {r["Name"][:70]}')
PY
done
